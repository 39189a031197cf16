"""Diagnostic: is there a synthetic configuration whose PSNR plateaus within a
few thousand steps, where the member-to-member spread collapses?  HIP side only (the product
Trainer, psnr_trajectory.run_hip): for each target variant, M members (own init, batches, noise,
refresh seeds) trained STEPS steps on its own batch sequence (drawn by PROCS worker processes
before the run: ~30 ms per 2048-ray batch on the host) or, with PLATEAU_POOL > 0, on a pool of that
many batches cycled, PSNR on the held-out rays every EVERY steps.  Prints one JSON line per
(variant, member) and a summary (mean, sd across members, run-to-run sd) per checkpoint."""
import json
import math
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import psnr_trajectory as pt  # noqa: E402

VARIANTS = os.environ.get("PLATEAU_GT", "surface_bright,surface_smooth,surface_flat").split(",")
MEMBERS = int(os.environ.get("PLATEAU_MEMBERS", "4"))
MEMBER0 = int(os.environ.get("PLATEAU_MEMBER0", "0"))  # first member index (extending an ensemble)
STEPS = int(os.environ.get("PLATEAU_STEPS", "3000"))
EVERY = int(os.environ.get("PLATEAU_EVERY", "250"))
POOL = int(os.environ.get("PLATEAU_POOL", "0"))  # 0: fresh batches every step (drawn in parallel)
PROCS = int(os.environ.get("PLATEAU_PROCS", "12"))
RAYS = int(os.environ.get("PLATEAU_RAYS", "2048"))
REPEATS = int(os.environ.get("PLATEAU_REPEATS", "2"))


_SCENE = None


def _draw(args):
    global _SCENE
    gt, k, m = args
    if _SCENE is None:
        from ncnerf_amd.synthetic import SyntheticScene
        _SCENE = SyntheticScene()
    return _SCENE.batch(RAYS, seed=pt.batch_seed(k, m), gt=gt)


class Cycle:
    def __init__(self, pool):
        self.pool = pool

    def __getitem__(self, k):
        return self.pool[k % len(self.pool)]


def main():
    from ncnerf_amd.synthetic import SyntheticScene
    scene = SyntheticScene()
    # every member's batch sequence is drawn first, by spawned worker processes (none of them, nor this
    # process yet, has touched the GPU)
    seqs = {}
    if not POOL:
        import multiprocessing as mp
        with mp.get_context("spawn").Pool(PROCS) as pp:
            for gt in VARIANTS:
                for m in range(MEMBER0, MEMBER0 + MEMBERS):
                    seqs[gt, m] = pp.map(_draw, [(gt, k, m) for k in range(STEPS)], chunksize=32)
                    print(json.dumps({"drawn": gt, "member": m}), flush=True)
    out = {}
    for gt in VARIANTS:
        pt.GT = gt
        curves = {}
        for m in range(MEMBER0, MEMBER0 + MEMBERS):
            t0 = time.time()
            if POOL:
                batches = Cycle([scene.batch(RAYS, seed=pt.batch_seed(k, m), gt=gt) for k in range(POOL)])
            else:
                batches = seqs.pop((gt, m))
            runs = []
            for r in range(REPEATS):
                res = pt.run_hip(STEPS, EVERY, lambda s: None, member=m, n_rays=RAYS, batches=batches)
                runs.append([c["psnr"] for c in res["curve"]])
            curves[m] = runs
            print(json.dumps({"gt": gt, "member": m, "psnr": runs, "t_s": round(time.time() - t0, 1)}), flush=True)
        steps = list(range(EVERY, STEPS + 1, EVERY))
        summ = []
        for i, st in enumerate(steps):
            means = [sum(r[i] for r in curves[m]) / len(curves[m]) for m in curves]
            mu = sum(means) / len(means)
            sd = math.sqrt(sum((x - mu) ** 2 for x in means) / max(len(means) - 1, 1))
            rr = [abs(curves[m][0][i] - curves[m][1][i]) / math.sqrt(2) for m in curves] if REPEATS > 1 else []
            summ.append({"step": st, "mean": round(mu, 3), "member_sd": round(sd, 3),
                         "run_to_run_sd": round(math.sqrt(sum(x * x for x in rr) / len(rr)), 3) if rr else None})
        out[gt] = summ
        print(json.dumps({"gt": gt, "summary": summ}), flush=True)
    print(json.dumps({"plateau_probe": out, "members": MEMBERS, "rays": RAYS, "pool": POOL}))


if __name__ == "__main__":
    main()
