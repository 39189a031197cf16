"""Summarise tools/eval_render_probe.py's rocprofv3 kernel trace: per image (between the spin
markers) the kernel span, the GPU-busy time (union of kernel intervals), the number of kernels and
the busy share of the wall time the probe printed.
python3 tools/eval_render_summary.py <kernel_trace.csv> <probe json line file> > profiles/<round>/eval_render_timeline.json"""
import csv
import json
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
probe = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
marks = [i for i, r in enumerate(rows) if "sleep" in r["Kernel_Name"].lower() or "spin" in r["Kernel_Name"].lower()]
out = []
for n, (a, b) in enumerate(zip(marks[-len(probe["images"]) - 1:-1], marks[-len(probe["images"]):])):
    seg = rows[a + 1:b]
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in seg)
    busy, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    span = (iv[-1][1] - iv[0][0]) / 1e3 if iv else 0.0
    kinds = {}
    for r in seg:
        k = r["Kernel_Name"].split("(")[0][:60]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        kinds.setdefault(k, [0, 0.0])
        kinds[k][0] += 1
        kinds[k][1] += d
    img = probe["images"][n]
    top = sorted(kinds.items(), key=lambda kv: -kv[1][1])[:8]
    out.append({"cam": img["cam"], "wall_ms": img["wall_ms"], "kernel_span_ms": round(span / 1e3, 3),
                "gpu_busy_ms": round(busy / 1e6, 3), "busy_share_of_wall": round(busy / 1e6 / img["wall_ms"], 3),
                "kernels": len(seg), "loop_iterations": img.get("iterations"),
                "host_blocked_ms": round(1e3 * img.get("blocked_s", 0.0), 3),
                "top_kernels_us": {k: [c, round(t, 1)] for k, (c, t) in top}})
print(json.dumps({"source": "rocprofv3 --kernel-trace over tools/eval_render_probe.py", "images": out}, indent=1))
