"""Paired PSNR comparison at the plateau: the HIP members of
tools/plateau_probe.py (one log line per member: R runs x checkpoints) against the oracle members
of tests/psnr_trajectory.py ref (one JSON per member), paired by member (same init, batches, noise
and refresh seeds).  Per checkpoint: the oracle and HIP means, the paired difference
d_m = mean_r(HIP_m,r) - oracle_m with its standard error and 95 % interval (t, M - 1 dof), the
member spread and the HIP run-to-run sd.

Usage: python tools/plateau_compare.py HIP_LOG[,HIP_LOG...] ORACLE_DIR [--json OUT]"""
import glob
import json
import math
import os
import sys

T975 = {1: 12.706, 2: 4.303, 3: 3.182, 4: 2.776, 5: 2.571, 6: 2.447, 7: 2.365, 8: 2.306, 9: 2.262, 10: 2.228,
        11: 2.201, 12: 2.179, 15: 2.131, 20: 2.086, 30: 2.042}


def t975(dof):
    return T975.get(dof) or T975[min(T975, key=lambda k: abs(k - dof))]


def main():
    hip_log, odir = sys.argv[1], sys.argv[2]
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    hip, gt, every = {}, None, None
    for path in hip_log.split(","):  # (several logs: an ensemble extended by later runs)
        for line in open(path):
            if not line.startswith("{"):
                continue
            r = json.loads(line)
            if "member" in r and "psnr" in r:
                hip[r["member"]] = r["psnr"]
                gt = r["gt"]
    orc = {}
    for f in sorted(glob.glob(os.path.join(odir, "member*.json"))):
        d = json.load(open(f))
        if gt is not None and d.get("gt") != gt:
            continue
        orc[d["member"]] = {c["step"]: c["psnr"] for c in d["curve"]}
    members = sorted(set(hip) & set(orc))
    n_ck = min(len(hip[m][0]) for m in members)
    steps_all = sorted(set.intersection(*[set(orc[m]) for m in members]))
    every = steps_all[0] if steps_all else 250
    rows = []
    for i in range(n_ck):
        st = every * (i + 1)
        if any(st not in orc[m] for m in members):
            continue
        h = [sum(run[i] for run in hip[m]) / len(hip[m]) for m in members]
        o = [orc[m][st] for m in members]
        d = [a - b for a, b in zip(h, o)]
        M = len(d)
        md = sum(d) / M
        sd = math.sqrt(sum((x - md) ** 2 for x in d) / max(M - 1, 1))
        se = sd / math.sqrt(M)
        rr = []
        for m in members:
            runs = [run[i] for run in hip[m]]
            mu = sum(runs) / len(runs)
            if len(runs) > 1:
                rr.append(sum((x - mu) ** 2 for x in runs) / (len(runs) - 1))
        mo, mh = sum(o) / M, sum(h) / M
        rows.append({"step": st, "members": M, "oracle_mean": round(mo, 3), "hip_mean": round(mh, 3),
                     "paired_delta": round(md, 3), "se": round(se, 3),
                     "ci95": [round(md - t975(M - 1) * se, 3), round(md + t975(M - 1) * se, 3)],
                     "sd_of_d": round(sd, 3),
                     "oracle_member_sd": round(math.sqrt(sum((x - mo) ** 2 for x in o) / max(M - 1, 1)), 3),
                     "hip_run_to_run_sd": round(math.sqrt(sum(rr) / len(rr)), 3) if rr else None})
    res = {"gt": gt, "members": members, "hip_runs_per_member": len(hip[members[0]]), "rows": rows}
    print("| step | M | oracle mean | HIP mean | paired Δ ± SE (dB) | 95 % CI | sd of d_m | oracle member sd | HIP run-to-run sd |")
    print("|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['step']} | {r['members']} | {r['oracle_mean']:.3f} | {r['hip_mean']:.3f} | {r['paired_delta']:+.3f} ± "
              f"{r['se']:.3f} | [{r['ci95'][0]:+.3f}, {r['ci95'][1]:+.3f}] | {r['sd_of_d']:.3f} | {r['oracle_member_sd']:.3f} | "
              f"{r['hip_run_to_run_sd']} |")
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
