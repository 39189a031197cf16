"""Summarise tools/profile_round.sh output (gpurun_out/prof_round) into profiles/<round>/:
kernel_stats.csv (rocprofv3 --stats of the bench), composite_fw_traffic.json (per-dispatch median
of FETCH_SIZE x2 + WRITE_SIZE for the composite forward; the x2 is the gfx950 FETCH_SIZE correction
of MI355X_MICROARCH.md's HBM section)."""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", "prof_round")


def counter_values(counter, kernel_sub):
    files = glob.glob(os.path.join(SRC, counter, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if kernel_sub in row["Kernel_Name"] and row["Counter_Name"] == counter:
                key = (f, row["Dispatch_Id"])
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main(rnd):
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(SRC, "trace", "**", "*kernel_stats.csv"), recursive=True)
    shutil.copy(stats[0], os.path.join(dst, "kernel_stats.csv"))
    k = "composite_fw_kernel"
    fetch, write = counter_values("FETCH_SIZE", k), counter_values("WRITE_SIZE", k)
    fm, wm = statistics.median(fetch), statistics.median(write)
    out = {"kernel": k, "traffic_bytes_per_launch": int(round((2 * fm + wm) * 1024)),
           "FETCH_SIZE_kb_median": fm, "WRITE_SIZE_kb_median": wm, "dispatches": len(fetch),
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over `bench.py --steps 5` "
                     "(graph replays + eager pass + roofline launches), per-dispatch median; gfx950 correction: "
                     "FETCH_SIZE x2 (MI355X_MICROARCH.md HBM), WRITE_SIZE as read; Infinity-Cache hits included"}
    json.dump(out, open(os.path.join(dst, "composite_fw_traffic.json"), "w"), indent=1)
    print(json.dumps(out))
    # bench.py's roofline launches are the last 135 composite_fw dispatches of the traced run (24 first
    # calls, 48 cycling 24 input sets = HBM-cold, 48 on one set = warm, 3 first calls + 12 over the
    # 65536-ray sets); in-step = the dispatches right behind a field forward.  The rocprof averages
    # must agree with bench.py's live HIP-event figures (roofline.avg_launch_us / warm_us).
    traces = glob.glob(os.path.join(SRC, "trace", "**", "*kernel_trace.csv"), recursive=True)
    rows = sorted(csv.DictReader(open(traces[0])), key=lambda r: int(r["Start_Timestamp"]))
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0  # noqa: E731
    d = [dur(r) for r in rows if k in r["Kernel_Name"]]
    instep = [dur(r) for i, r in enumerate(rows) if k in r["Kernel_Name"] and i and "field_fwd" in rows[i - 1]["Kernel_Name"]]
    rest = d[:-135]
    live = {"kernel": k + "<3> (ncn_composite_train_fw_bg)",
            "source": "rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 30 --no-cpu-baseline "
                      "--no-bf16-line --no-extra-states (gpurun_out/prof_round/trace)",
            "hbm_cold_48_launches_avg_us": round(statistics.mean(d[-111:-63]), 3),
            "warm_48_launches_avg_us": round(statistics.mean(d[-63:-15]), 3),
            "batch65536_12_launches_avg_us": round(statistics.mean(d[-12:]), 3),
            "in_step_avg_us": round(statistics.mean(instep), 3), "in_step_median_us": round(statistics.median(instep), 3),
            "in_step_dispatches": len(instep),
            "in_step_and_eager_avg_us": round(statistics.mean(rest), 3), "in_step_and_eager_dispatches": len(rest),
            "note": "the bench's roofline launches are the last 135 dispatches: 24 first calls, 48 cycling 24 input "
                    "sets (HBM-cold), 48 on one set (warm), 3 first calls + 12 over the 65536-ray sets; in_step = the "
                    "dispatches right behind a field_fwd (graph-replayed steps and the bench's in-step probe); the "
                    "rocprof kernel durations exclude the per-launch gaps that bench.py's event pair around the "
                    "back-to-back launches includes"}
    json.dump(live, open(os.path.join(dst, "composite_fw_rocprof_timing.json"), "w"), indent=1)
    print(json.dumps(live))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "round1")
