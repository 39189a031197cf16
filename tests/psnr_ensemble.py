"""PSNR parity as an ENSEMBLE statistic (VERDICT r2 "do this" 1) — test infrastructure.

Single training trajectories on this synthetic room are chaotic (two HIP runs on identical inputs
split by several dB once one of them breaks through a plateau), so parity after equal steps is
measured over seed ensembles on both sides:
  * oracle side (CPU, slow, committed as the fixture tests/golden/psnr_oracle_ensemble.json):
      python tests/psnr_trajectory.py ref --member m --rays 2048 --steps 1000 --every 125 --impl c
    for members m = 0..M-1, then  python tests/psnr_ensemble.py merge <files...>;
  * HIP side (GPU):  python tests/psnr_ensemble.py hip --repeats R --out profiles/<round>/psnr_ensemble.json
  * offline:  python tests/psnr_ensemble.py compare A.json B.json [--out C.json] — A (a HIP output or
    another oracle ensemble) against the oracle ensemble B, paired by member
    member m with the same initial parameters, batches, marcher noise and refresh seeds, R runs
    each (they differ only by the float-atomic order of the table-gradient flush).
Statistics per checkpoint: the mean PSNR and its standard error on each side (HIP: the mean of a
member's runs is one sample), the paired difference d_m = HIP_m - oracle_m (mean, SE, 95 % CI)
and the within-member HIP spread (the chaos floor a single pair is read against).
"""
import argparse
import json
import math
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

FIXTURE = os.path.join(HERE, "golden", "psnr_oracle_ensemble.json")
T95 = {2: 12.71, 3: 4.30, 4: 3.18, 5: 2.78, 6: 2.57, 7: 2.45, 8: 2.36, 9: 2.31, 10: 2.26, 11: 2.23, 12: 2.20,
       13: 2.18, 14: 2.16, 15: 2.14, 16: 2.13}


def mean_se(xs):
    n = len(xs)
    m = sum(xs) / n
    if n < 2:
        return m, float("nan"), 0.0
    sd = math.sqrt(sum((x - m) ** 2 for x in xs) / (n - 1))
    return m, sd / math.sqrt(n), sd


def merge(files, out=FIXTURE):
    members = []
    for f in files:
        r = json.load(open(f))
        members.append({"member": r["member"], "init_seed": r["init_seed"], "rays_per_step": r["rays_per_step"],
                        "steps": r["steps"], "curve": [{"step": c["step"], "psnr": round(c["psnr"], 5),
                                                        "loss": round(c["loss"], 7)} for c in r["curve"]]})
    members.sort(key=lambda m: m["member"])
    first = json.load(open(files[0]))
    preset = first.get("preset", "hypersim")
    emulate, emulate_bwd = first.get("emulate"), bool(first.get("emulate_bwd"))
    sampling = first.get("grid_sampling", "device")
    flags = ((f" --emulate {emulate}" if emulate else "") + (" --emulate-bwd" if emulate_bwd else "")
             + ("" if sampling == "device" else f" --sampling {sampling}")
             + ("" if preset == "hypersim" else f" --preset {preset}"))
    side = ("oracle CPU (fp32), oracle/train_ref.py with the C hash-grid statement" if not emulate else
            f"oracle CPU, oracle/train_ref.py with the C hash-grid statement, MLP operands rounded to {emulate}"
            + (" and the field backward's loss-scaled fp16 gradient chain emulated (GradScaler)" if emulate_bwd else "")
            + f"; grid refresh sampling: {sampling}")
    res = {"side": side, "gt": "surface_bright", "eval_rays": 16384, "members": members, "preset": preset,
           "emulate": emulate, "emulate_bwd": emulate_bwd, "grid_sampling": sampling,
           "generator": "python tests/psnr_trajectory.py ref --member m --rays 2048 --steps 1000 --every 125 --impl c"
                        + flags}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(f"{out}: {len(members)} members")


def stats(oracle, hip_runs):
    """oracle: fixture dict; hip_runs: {member: [curve, ...]} -> per-step statistics."""
    om = {m["member"]: {c["step"]: c["psnr"] for c in m["curve"]} for m in oracle["members"]}
    steps = sorted(set.intersection(*[set(v) for v in om.values()]))
    out = []
    for st in steps:
        mem = [m for m in om if m in hip_runs and all(any(c["step"] == st for c in r) for r in hip_runs[m])]
        if not mem:
            continue
        hip_m = {m: [next(c["psnr"] for c in r if c["step"] == st) for r in hip_runs[m]] for m in mem}
        h = [sum(v) / len(v) for v in hip_m.values()]
        o = [om[m][st] for m in mem]
        d = [a - b for a, b in zip(h, o)]
        hm, hse, _ = mean_se(h)
        omn, ose, _ = mean_se(o)
        dm, dse, dsd = mean_se(d)
        within = [mean_se(v)[2] for v in hip_m.values() if len(v) > 1]
        t = T95.get(len(d), 2.0)
        out.append({"step": st, "members": len(mem), "hip_mean": round(hm, 4), "hip_se": round(hse, 4),
                    "oracle_mean": round(omn, 4), "oracle_se": round(ose, 4), "paired_delta_mean": round(dm, 4),
                    "paired_delta_se": round(dse, 4), "paired_delta_ci95": [round(dm - t * dse, 4), round(dm + t * dse, 4)],
                    "paired_delta_sd": round(dsd, 4),
                    "hip_within_member_sd": round(sum(within) / len(within), 4) if within else None})
    return out


def run_hip_ensemble(members, repeats, steps, every, n_rays, log, preset="hypersim"):
    import psnr_trajectory as pt
    runs = {}
    for m in members:
        batches = pt.host_batches(steps, n_rays, m)
        runs[m] = []
        for r in range(repeats):
            t0 = time.time()
            res = pt.run_hip(steps, every, lambda s: None, member=m, n_rays=n_rays, batches=batches,
                             trainer_kw={"preset": preset})
            runs[m].append(res["curve"])
            log(f"member {m} run {r}: " + " ".join(f"{c['step']}:{c['psnr']:.3f}" for c in res["curve"])
                + f" ({time.time() - t0:.1f} s)")
    return runs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("merge", "hip", "compare"))
    ap.add_argument("files", nargs="*")
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--members", type=int, default=None, help="(hip) first M members of the fixture")
    ap.add_argument("--steps", type=int, default=None, help="(hip) default: the fixture's")
    ap.add_argument("--out", default=None)
    ap.add_argument("--fixture", default=FIXTURE, help="the oracle ensemble (merge: output; hip: input)")
    a = ap.parse_args()
    if a.mode == "merge":
        merge(a.files, a.out or a.fixture)
        return
    if a.mode == "compare":
        # compare A B: paired statistics of A (a hip ensemble output, or an oracle ensemble fixture
        # taken as one run per member) against the oracle ensemble B, offline
        ra, ob = json.load(open(a.files[0])), json.load(open(a.files[1]))
        if "hip_runs" in ra:
            runs = {int(k): v for k, v in ra["hip_runs"].items()}
        else:
            runs = {m["member"]: [m["curve"]] for m in ra["members"]}
        st = stats(ob, runs)
        for s in st:
            print(json.dumps(s))
        if a.out:
            with open(a.out, "w") as f:
                json.dump({"a": a.files[0], "b": a.files[1], "stats": st}, f, indent=1)
        return
    log = lambda s: print(s, flush=True)  # noqa: E731
    oracle = json.load(open(a.fixture))
    mems = [m["member"] for m in oracle["members"]][: a.members]
    steps = a.steps or oracle["members"][0]["steps"]
    n_rays = oracle["members"][0]["rays_per_step"]
    every = oracle["members"][0]["curve"][0]["step"]
    runs = run_hip_ensemble(mems, a.repeats, steps, every, n_rays, log, oracle.get("preset", "hypersim"))
    st = stats(oracle, runs)
    for s in st:
        log(json.dumps(s))
    res = {"rays_per_step": n_rays, "steps": steps, "repeats": a.repeats, "members": mems, "stats": st,
           "hip_runs": {str(k): v for k, v in runs.items()}}
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
