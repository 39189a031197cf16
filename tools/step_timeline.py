"""Print one graph-replayed training step (and one grid-refresh step) from a rocprofv3 kernel trace:
python3 tools/step_timeline.py gpurun_out/<dir>/run_kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "adam_apply" in r["Kernel_Name"]]


def show(seg, t0):
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1000:8.1f} {(e - s) / 1000:7.1f}  {r['Kernel_Name'][:80]}")
    print("span us", (int(seg[-1]["End_Timestamp"]) - t0) / 1000)


done = set()
for j in range(len(ends) - 1, 0, -1):
    seg = rows[ends[j - 1] + 1:ends[j] + 1]
    kind = "refresh" if any("grid_select" in r["Kernel_Name"] for r in seg) else "step"
    if any("spin" in r["Kernel_Name"] for r in seg) or kind in done:
        continue
    print(f"--- {kind}")
    show(seg, int(rows[ends[j - 1]]["End_Timestamp"]))
    done.add(kind)
    if len(done) == 2:
        break
