"""Print one graph-replayed training step (and one grid-refresh step) from a rocprofv3 kernel trace:
python3 tools/step_timeline.py gpurun_out/<dir>/run_kernel_trace.csv
A step runs from one ncn_step_inputs launch to the next (with the deferred optimizer, the previous
step's Adam runs on a side stream inside it, beside the marcher)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "step_inputs_kernel" in r["Kernel_Name"]]


def show(seg, t0):
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1000:8.1f} {(e - s) / 1000:7.1f}  {r['Kernel_Name'][:80]}")
    print("span us", (max(int(r["End_Timestamp"]) for r in seg) - t0) / 1000)


done = set()
for j in range(len(starts) - 2, 0, -1):
    seg = rows[starts[j]:starts[j + 1]]
    kind = "refresh" if any("grid_select" in r["Kernel_Name"] for r in seg) else "step"
    if any("spin" in r["Kernel_Name"] for r in seg) or kind in done:
        continue
    print(f"--- {kind}")
    show(seg, int(seg[0]["Start_Timestamp"]))
    done.add(kind)
    if len(done) == 2:
        break

# per-kernel medians over every graph-replayed training step of the trace (one step's timeline above
# is a single sample; the kernels vary by a few percent from step to step)
import statistics  # noqa: E402

per, spans = {}, []
for j in range(len(starts) - 1):
    seg = rows[starts[j]:starts[j + 1]]
    if any("grid_select" in r["Kernel_Name"] or "spin" in r["Kernel_Name"] for r in seg):
        continue
    names = [r["Kernel_Name"] for r in seg]
    if not any("field_scatter" in nm for nm in names):
        continue
    t0 = int(seg[0]["Start_Timestamp"])
    spans.append((max(int(r["End_Timestamp"]) for r in seg) - t0) / 1000)
    seen = {}
    for r in seg:
        k = r["Kernel_Name"][:80]
        seen[k] = seen.get(k, 0) + 1
        per.setdefault((k, seen[k]), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
print(f"--- medians over {len(spans)} training steps (us): span median {statistics.median(spans):.1f}")
for (k, i), v in per.items():
    if len(v) >= len(spans) // 2:
        print(f"{statistics.median(v):8.1f}  (p10 {sorted(v)[len(v) // 10]:.1f}, p90 {sorted(v)[(9 * len(v)) // 10]:.1f})  {k}")
