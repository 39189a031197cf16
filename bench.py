"""Training-throughput benchmark of the HIP hot path (BASELINE.json metric: training rays/s +
samples/s at 1/2/4/8 GPUs).

Workload (BASELINE.json configs[1] + [2]): one full training step per iteration on a synthetic
Hypersim-shaped batch of 8192 rays per GPU (128 random 8x8 patches, ai_001_001 scene box,
procedural room occupancy): ray/AABB -> occupancy-grid march -> fused hash-grid +
MLP field -> composite -> rgb/opacity/normal-clustering losses -> backward -> [RCCL all-reduce of
the flat gradient] -> clip + Adam, and the occupancy-grid refresh every 16 steps.  Inputs are
generated on the device before the timed region.  N>1: one process per GPU (torchrun), weak
scaling (8192 rays per rank), value = all ranks' rays / max-over-ranks time.

Launch: under torchrun (WORLD_SIZE set) every process is one rank; `--gpus N` with N > 1 and no
WORLD_SIZE spawns the N local ranks itself (child processes with RANK/LOCAL_RANK/WORLD_SIZE and a
127.0.0.1 rendezvous, started before this process touches the GPU) and exits with the worst child
status.  Either way the run fails unless the process group has exactly --gpus ranks.

Prints ONE JSON line on rank 0.
"""
import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv):
    """Start n local ranks of this script (no GPU call has happened in this process) and return the
    worst exit status.  Rank 0's stdout (the JSON line) passes through; the others' is discarded."""
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    # poll every rank: the first non-zero exit ends the others (a crashed rank would otherwise leave
    # its peers blocked in a collective and this parent waiting on them forever)
    import time
    rc = 0
    while any(p.poll() is None for p in procs):
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad:
            rc = bad[0]
            break
        time.sleep(0.2)
    for p in procs:
        if p.poll() is None:
            p.terminate()
    for p in procs:
        try:
            p.wait(timeout=20)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
        rc = rc or p.returncode
    return rc


if __name__ == "__main__" and "WORLD_SIZE" not in os.environ:
    _gpus = 1
    for _i, _a in enumerate(sys.argv):
        if _a == "--gpus" and _i + 1 < len(sys.argv):
            _gpus = int(sys.argv[_i + 1])
        elif _a.startswith("--gpus="):
            _gpus = int(_a.split("=", 1)[1])
    if _gpus > 1:
        sys.exit(spawn_ranks(_gpus, sys.argv[1:]))

import math  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, spec)
HBM_COPY_GBS = 6290.0  # MI355X_MICROARCH.md: float4 copy, measured (79 % of the spec)
TIMED = ("ncn_composite_train_fw_bg", "ncn_composite_train_bw_bg", "ncn_march_train_fused", "ncn_field_fwd",
         "ncn_field_bwd", "ncn_field_bwd_mlp_part", "ncn_field_scatter", "ncn_field_scatter_wgrad", "ncn_cluster_loss")


def window_start(base, warmup, steps, every=16):
    """The first global step (>= base) of the warm-up + timed steps whose timed window holds the
    long-run share of grid refreshes, round(steps / every) of the global steps that are multiples
    of `every` (Trainer.update_interval: train_nerf.py:318 refreshes every 16 steps).  Without it a
    window's count depends on where it falls: 20 steps from 3005 held two refreshes (one per 10
    steps instead of one per 16).  Returns (step0, refreshes in the timed window)."""
    want = int(steps / every + 0.5)
    count = lambda a: (a + steps - 1) // every - (a - 1) // every  # noqa: E731
    for s0 in range(base, base + every):
        if count(s0 + warmup) == want:
            return s0, want
    return base, count(base + warmup)


def pmc_traffic():
    """HBM bytes per composite_fw launch from the committed rocprofv3 PMC summary (FETCH_SIZE x2 +
    WRITE_SIZE, separate passes; profiles/<round>/composite_fw_traffic.json), or None."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "composite_fw_traffic.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    return d.get("traffic_bytes_per_launch"), os.path.relpath(files[-1], ROOT)


def composite_fw_roofline(model, batches, dev, scene_big, reps=48, n_sets=24):
    """Live HIP-event measurement of the roofline kernel, the training step's compositor
    (ncn_composite_train_fw_bg over the fused marcher's rays_a, long rays first).  `n_sets` input
    sets (the bench batches marched with different jitter and run through the field as in the step,
    ~16.5 MB each: 24 sets ~ 400 MB, ~1.5x the 256 MiB Infinity Cache) are prepared; then
      hbm:     `reps` back-to-back launches cycling through the sets behind a GPU spin: every launch
               reads inputs the launches between evicted from the caches (HBM-bound), the average
               launch duration -> `achieved` / `frac`;
      warm:    `reps` back-to-back launches on ONE set (its inputs cache-resident);
      in_step: one launch right behind the field forward that wrote its inputs, bracketed by its own
               event pair (includes the launch ramp and the event overhead), mean over the batches.
    Returns (algorithmic bytes per launch (mean over the sets), {hbm, warm, in_step, ...} us)."""
    from ncnerf_amd import _lib
    from ncnerf_amd._lib import F32, I32, I64, ptr, stream
    from ncnerf_amd import vren
    from ncnerf_amd.rendering import march_buffers, march_train_fused
    fn = _lib.lib().ncn_composite_train_fw_bg  # the step's compositor (ray-major)
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

    def rm_args(k, R, S):
        return [ptr(k["sig"]), ptr(k["rgb"]), ptr(k["dl"]), ptr(k["ts"]), ptr(k["ra"]), I64(R), I64(S), I32(3),
                F32(1e-4)] + [ptr(t) for t in k["res"][:5]] + [F32(1.0), ptr(k["res"][5]), stream()]

    sets, t_in = [], []
    with torch.no_grad():
        for j in range(n_sets):
            batch = batches[j % len(batches)]
            o, d = batch["rays_o"].contiguous(), batch["rays_d"].contiguous()
            R = o.shape[0]
            mk = march_train_fused(model, o, d, 0.01, 1024, noise=torch.rand(R, device=dev),
                                   out=march_buffers(R, 1024, dev))
            S = int(mk["counter"][0].item())
            out = model(mk["xyzs"], mk["dirs"], n_samples_dev=mk["counter"])
            res = [torch.empty(R, dtype=torch.int64, device=dev), torch.empty(R, device=dev), torch.empty(R, device=dev),
                   torch.empty(R, 3, device=dev), torch.empty(S, device=dev), torch.empty(R, 3, device=dev)]
            if j < len(batches):  # in-step: right behind the field forward that produced the inputs, as
                # the step launches it (capacity-sized arrays)
                full = {"sig": out["sigmas"], "rgb": out["rgbs"], "dl": mk["deltas"], "ts": mk["ts"],
                        "ra": mk["rays_a"],
                        "res": res[:4] + [torch.empty(mk["ts"].shape[0], device=dev), res[5]]}
                args = rm_args(full, R, mk["ts"].shape[0])
                for rep in range(2):  # (rep 0 warms up)
                    if rep:
                        out = model(mk["xyzs"], mk["dirs"], n_samples_dev=mk["counter"])
                    a, b = ev(), ev()
                    a.record()
                    assert fn(*args) == 0
                    b.record()
                    torch.cuda.synchronize()
                t_in.append(a.elapsed_time(b) * 1e3)
                del full
            # compact copies (S rows) so the sets are disjoint, cache-sized data
            keep = {"sig": out["sigmas"][:S].clone(), "rgb": out["rgbs"][:S].clone(), "dl": mk["deltas"][:S].clone(),
                    "ts": mk["ts"][:S].clone(), "ra": mk["rays_a"].clone(), "res": res}
            keep["args"] = rm_args(keep, R, S)
            sets.append(keep)
            del out, mk
        for k in sets:  # (first-call costs, and the algorithmic bytes of each set)
            assert fn(*k["args"]) == 0
        torch.cuda.synchronize()
        nbytes = [24.0 * float(k["res"][0].sum().item()) + 4.0 * k["sig"].shape[0] + 52.0 * k["ra"].shape[0]
                  for k in sets]

        def b2b(f, arg_list, n=reps):
            torch.cuda.synchronize()
            a, b = ev(), ev()
            torch.cuda._sleep(2_000_000)  # ~1 ms: every launch below is queued before the first runs
            a.record()
            for i in range(n):
                f(*arg_list[i % len(arg_list)])
            b.record()
            torch.cuda.synchronize()
            return a.elapsed_time(b) * 1e3 / n

        t_hbm = b2b(fn, [k["args"] for k in sets])
        t_warm = b2b(fn, [sets[0]["args"]])
        # the same kernel on config #4's global batch (65536 rays, one launch): 3 sets of ~140 MB
        # cycled (> the Infinity Cache), so each launch reads from HBM
        big = []
        for j in range(3):
            b = scene_big.torch_batch(65536, seed=777 + j, device=dev)
            o, d = b["rays_o"].contiguous(), b["rays_d"].contiguous()
            # (the reference's 3-call marcher API: the one-launch marcher takes <= 16384 rays)
            _, ht, _ = vren.ray_aabb_intersect(o, d, model.center, model.half_size, 1, near_distance=0.01)
            ra, xyzs, dirs, deltas, ts, counter = vren.raymarching_train(
                o, d, ht[:, 0].contiguous(), model.density_bitfield, 1, 0.5, 0.0, torch.rand(65536, device=dev), 128,
                1024)
            S = int(counter[0].item())
            # rows as the training step's marcher orders them (march_train_place): rays longer than
            # 256 samples first, the rest in ray order (sample segments unchanged)
            long_ = ra[:, 2] > 256
            ra = torch.cat([ra[long_], ra[~long_]]).contiguous()
            out = model(xyzs, dirs)
            R = 65536
            res = [torch.empty(R, dtype=torch.int64, device=dev), torch.empty(R, device=dev), torch.empty(R, device=dev),
                   torch.empty(R, 3, device=dev), torch.empty(S, device=dev), torch.empty(R, 3, device=dev)]
            k = {"sig": out["sigmas"][:S].clone(), "rgb": out["rgbs"][:S].clone(), "dl": deltas[:S].clone(),
                 "ts": ts[:S].clone(), "ra": ra.clone(), "res": res}
            k["args"] = rm_args(k, R, S)
            del out
            big.append(k)
        for k in big:
            assert fn(*k["args"]) == 0
        torch.cuda.synchronize()
        big_bytes = [24.0 * float(k["res"][0].sum().item()) + 4.0 * k["sig"].shape[0] + 52.0 * k["ra"].shape[0]
                     for k in big]
        t_big = b2b(fn, [k["args"] for k in big], n=12)
        del big
    mean_bytes = float(np.mean([nbytes[i % len(sets)] for i in range(reps)]))
    return mean_bytes, {"hbm": t_hbm, "warm": t_warm, "in_step": float(np.mean(t_in)), "warm_bytes": nbytes[0],
                        "big_us": t_big,
                        "big_bytes": float(np.mean(big_bytes))}


def _cpu_leg(threads, n_rays, steps, warmup, budget_s=30.0):
    from oracle.train_ref import CPUTrainer
    from ncnerf_amd.synthetic import SyntheticScene
    torch.set_num_threads(threads)
    scene = SyntheticScene()
    tr = CPUTrainer(scene.bitfield)
    for k in range(warmup):
        t0 = time.perf_counter()
        tr.step(scene.batch(n_rays, seed=999 + k))
        dt = time.perf_counter() - t0
        log(f"cpu leg ({threads} threads) warm-up step {k}: {1e3 * dt:.0f} ms")
        if dt > 15.0:
            return None, dt, 0  # oversubscribed (threads beyond the CPUs the process really gets)
    times = []
    for k in range(steps):
        b = scene.batch(n_rays, seed=k)
        t0 = time.perf_counter()
        tr.step(b)
        times.append(time.perf_counter() - t0)
        if k % 5 == 4:
            log(f"cpu leg ({threads} threads) step {k}: median {1e3 * float(np.median(times)):.0f} ms")
        if sum(times) > budget_s and len(times) >= 3:
            break  # bounded sample (an oversubscribed affinity mask can be far slower than the CPU share)
    return float(np.median(times)), float(sum(times)), len(times)


def distill_opaque(model, trainer, scene, dev, steps=300, n_points=1 << 16, sigma_in=3000.0, sigma_out=1e-2):
    """The opaque state of a converged NeRF, reached directly: the field's density is fitted to the
    procedural room's occupancy (log sigma -> log sigma_in inside occupied voxels, log sigma_out
    elsewhere; random points and directions, MSE on log sigma through the field backward and the
    trainer's own Adam), so that rays terminate at the first surface as they do once a scene's
    surfaces have converged (the photometric + opacity losses alone take far longer than the bench
    can spend to push T below 1e-4 on this room).  Returns the fit's last loss."""
    occ = torch.from_numpy(scene.occ).to(dev)
    G = occ.shape[0]
    g = torch.Generator(device=dev).manual_seed(77)
    lo, hi = math.log(sigma_out), math.log(sigma_in)
    loss = None
    for _ in range(steps):
        x = (torch.rand(n_points, 3, device=dev, generator=g) - 0.5) * 0.999
        v = ((x + 0.5) * G).long().clamp_(0, G - 1)
        target = torch.where(occ[v[:, 0], v[:, 1], v[:, 2]], hi, lo)
        d = torch.nn.functional.normalize(torch.randn(n_points, 3, device=dev, generator=g), dim=1)
        loss = ((torch.log(model(x, d)["sigmas"]) - target) ** 2).mean()
        loss.backward()
        trainer.opt.step()
    torch.cuda.synchronize()
    return round(float(loss.detach()), 4)


def cpu_quota():
    """CPUs of this process's cgroup CPU quota (cgroup v2 cpu.max, v1 cfs_quota_us), or None."""
    for path, split in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            text = open(path).read().strip()
            if split:
                q, p = split(text)
            else:
                q, p = text, open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read().strip()
            if q in ("max", "-1"):
                return None
            return max(1, math.ceil(int(q) / int(p)))
        except (OSError, ValueError):
            continue
    return None


def cpu_baseline(ray_counts=(2048, 8192), steps=20, warmup=3):
    """Oracle CPU port of the same step (pure PyTorch + C on the host cores) at config #1's 2048 rays
    and config #2's 8192 rays, timed as BASELINE.md §2 asks: median wall time of 20
    steps (fewer if a leg's timed steps pass 30 s) after 3 warm-up steps, on every CPU this process
    may use: one leg per distinct thread count among OMP_NUM_THREADS (the GPU box's CPU share) and
    the usable CPUs (the affinity mask capped by the cgroup CPU quota).  A thread count above the
    quota is skipped and reported (on the GPU box the mask holds 256 CPUs under a 16-CPU quota: 256
    threads took 80 s per step, round 4).  `value` is the fastest leg (the stronger baseline); every
    leg is reported."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    quota = cpu_quota()
    usable = min(affinity, quota) if quota else affinity
    threads_legs = {}
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < usable:
        threads_legs["omp_num_threads"] = int(omp)
    threads_legs["all_usable_cpus"] = usable
    runs, skipped = {}, {}
    if affinity > usable:
        skipped["affinity"] = f"{affinity} CPUs in the affinity mask > cgroup CPU quota {quota}: oversubscribed"
    for n_rays in ray_counts:
        for tname, threads in threads_legs.items():
            name = f"{tname}_{n_rays}_rays"
            med, tot, n = _cpu_leg(threads, n_rays, steps, warmup)
            if med is None:
                skipped[name] = f"{threads} threads: a warm-up step took {tot:.0f} s (oversubscribed); leg abandoned"
                log(f"cpu leg {name}: {skipped[name]}")
                continue
            log(f"cpu leg {name} ({threads} threads): {med * 1e3:.0f} ms/step")
            runs[name] = {"threads": threads, "rays_per_step": n_rays, "rays_per_s": round(n_rays / med, 1),
                          "ms_per_step": round(med * 1e3, 1), "timed_steps": n, "timed_s": round(tot, 1)}
    best = max(runs, key=lambda k: runs[k]["rays_per_s"])
    torch.set_num_threads(threads_legs.get("omp_num_threads", usable))
    return {"value": runs[best]["rays_per_s"], "unit": "rays/s", "cores": runs[best]["threads"], "kind": "port",
            "host_cpus": os.cpu_count(), "affinity_cpus": affinity, "cpu_quota": quota, "legs": runs,
            "skipped_legs": skipped,
            "sample": f"median of up to {steps} full training steps (at most ~30 s per leg) of "
                      + " and ".join(str(r) for r in ray_counts)
                      + f" rays (configs #1 / #2) after {warmup} warm-up steps on the oracle CPU path "
                      f"(oracle/train_ref.py: C marcher/compositor + torch fp32 field/losses), on all {usable} usable "
                      f"CPUs (min of affinity mask {affinity} and cgroup quota {quota})"
                      + (f" and on OMP_NUM_THREADS={threads_legs['omp_num_threads']}" if "omp_num_threads" in threads_legs
                         else "")
                      + f"; value = the fastest leg ({best})"}


def eval_render(model, scene, dev, n_images=3):
    """The test-time render of full 1024x768 images (786 432 rays each) through render(...,
    test_time=True): the reference's host-driven loop of rendering.py:45-149 (march N_samples per
    alive ray, field on the valid samples, incremental composite, alive compaction) with `model`.
    Wall time per image (synchronize on both sides), loop iterations, marched samples, and the host
    time blocked at the loop's per-iteration syncs (valid_mask.sum(), the alive compaction)."""
    from ncnerf_amd.rendering import render
    kw = dict(near_distance=0.01, max_samples=1024, test_time=True)
    res = []
    with torch.no_grad():
        o, d = scene.image_rays(0, dev)
        render(model, o, d, **kw)  # (first-call costs)
        for cam in range(1, n_images + 1):
            o, d = scene.image_rays(cam, dev)
            st = {}
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = render(model, o, d, loop_stats=st, **kw)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            res.append((t1 - t0, st, float(out["opacity"].mean())))
            log(f"eval_render image {cam}: {1e3 * (t1 - t0):.1f} ms, {st.get('iterations')} iterations")
    # the same images through the loop in the reference's structure (test_fused=False), for comparison
    ref_wall = []
    with torch.no_grad():
        o, d = scene.image_rays(0, dev)
        render(model, o, d, test_fused=False, **kw)  # (first-call costs of its torch ops)
        for cam in range(1, n_images + 1):
            o, d = scene.image_rays(cam, dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            render(model, o, d, test_fused=False, **kw)
            torch.cuda.synchronize()
            ref_wall.append(time.perf_counter() - t0)
            log(f"eval_render (reference loop) image {cam}: {1e3 * ref_wall[-1]:.1f} ms")
    wall = float(np.median([r[0] for r in res]))
    its = [r[1].get("iterations", 0) for r in res]
    blocked = [r[1].get("blocked_s", 0.0) / r[0] for r in res]
    return {"ms_per_image": round(wall * 1e3, 2), "rays_per_image": int(o.shape[0]),
            "rays_per_s": round(o.shape[0] / wall, 1), "images": n_images,
            "loop_iterations": its, "samples_marched_per_image": [int(r[1].get("samples_marched", 0)) for r in res],
            "host_blocked_share": round(float(np.median(blocked)), 3), "mean_opacity": [round(r[2], 3) for r in res],
            "reference_loop_ms_per_image": round(float(np.median(ref_wall)) * 1e3, 2),
            "method": "render(model, rays of one synthetic camera's full image, test_time=True): rendering.py:45-149's "
                      "loop on ncn_march_test / the field / ncn_composite_test_fw, fused iteration (the field over "
                      "the whole march output; reference_loop_ms_per_image: the loop in the reference's structure, "
                      "test_fused=False, bit-identical outputs); median wall time of "
                      f"{n_images} images after one warm-up image; host_blocked_share = host time inside the "
                      "loop's syncing statements / wall time"}


_T0 = time.time()


def log(msg):
    """Progress on stderr (the JSON line is the only stdout output)."""
    print(f"[bench {time.time() - _T0:7.1f} s] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rays", type=int, default=8192, help="rays per GPU per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-grid-update", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="eager (Python-launched) step instead of a HIP graph")
    ap.add_argument("--no-defer", action="store_true",
                    help="keep each step's optimizer at the end of its own graph (default: it runs in the next "
                         "step's graph beside the marcher, Trainer(defer_optimizer=True))")
    ap.add_argument("--no-split", action="store_true",
                    help="the autograd backward after the whole loss node (default: Trainer(split_backward=True), "
                         "the photometric backward beside the normal clustering)")
    ap.add_argument("--precision", choices=("fp16", "bf16"), default="fp16",
                    help="MFMA operand type of the field MLP (fp16 = tcnn's FullyFusedMLP, the reference's AMP run)")
    ap.add_argument("--no-bf16-line", action="store_true",
                    help="skip the second measurement of configs[2] with bf16 MLP operands")
    ap.add_argument("--pretrain", type=int, default=0,
                    help="untimed training steps from the random init before the warm-up, on the procedural "
                         "occupancy grid (not refreshed while pretraining); 0 (default) = the random-init weights "
                         "the contract asks for")
    ap.add_argument("--no-extra-states", action="store_true",
                    help="skip the extra measurements of trained states: 500 steps pretrained on the procedural "
                         "grid (rays terminate early), and the grid train_nerf.py maintains itself "
                         "(mark_invisible_cells + grid refresh from step 0)")
    ap.add_argument("--no-eval-render", action="store_true",
                    help="skip the test-time render of full 1024x768 images (eval_render line)")
    ap.add_argument("--dist-selftest", action="store_true",
                    help="launch/rendezvous check only (no GPU work): every rank all-reduces its rank, rank 0 "
                         "prints {world, backend, sum}")
    args = ap.parse_args()

    from ncnerf_amd import distributed

    rank, world = distributed.init_from_env()
    backend = dist.get_backend() if world > 1 else None
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the process group has {world} rank(s)", file=sys.stderr)
        sys.exit(3)
    if args.dist_selftest:
        if os.environ.get("NCN_SELFTEST_CRASH_RANK") == str(rank):  # (launch test: a rank that dies early)
            sys.exit(7)
        if os.environ.get("NCN_SELFTEST_HANG_RANK") == str(rank):  # (launch test: a rank that never returns)
            __import__("time").sleep(3600)
        t = torch.tensor([float(rank)])
        if world > 1:
            dist.all_reduce(t)
        if rank == 0:
            print(json.dumps({"world": world, "backend": backend, "rank_sum": float(t.item())}))
        if world > 1:
            dist.destroy_process_group()
        return

    from ncnerf_amd import _lib, synthetic
    from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers
    from ncnerf_amd.synthetic import SyntheticScene
    from ncnerf_amd.trainer import Trainer
    # (modulo: a 1-GPU rehearsal of the N>1 path with NCN_DIST_BACKEND=gloo puts every rank on cuda:0)
    local_rank = int(os.environ.get("LOCAL_RANK", 0)) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    torch.manual_seed(1234 + rank)

    GT = "surface_bright"  # synthetic target colours (ncnerf_amd.synthetic)

    def measure(precision, steps, kernel_table, pretrain, state="procedural", preset="hypersim"):
        """Build the model in `precision`, pretrain it `pretrain` untimed steps, warm up, time `steps`
        graph-replayed training steps (barrier + synchronize on both sides), max over ranks.
        state "procedural": the procedural occupancy grid, fixed while pretraining;
        "refreshed": mark_invisible_cells, then the grid refreshed from the model every 16 steps from
        step 0 (all cells for the first 256), as train_nerf.py does."""
        log(f"measure: {precision} {state} pretrain={pretrain} preset={preset}")
        scene = SyntheticScene()
        model = register_grid_buffers(NGPMT(scale=0.5, grid_size=128, precision=precision).to(dev))
        trainer = Trainer(model, update_grid=not args.no_grid_update, use_graph=not args.no_graph,
                          defer_optimizer=not args.no_defer, preset=preset, split_backward=not args.no_split)
        # marched / composited sample counts accumulated on the device by the step itself
        # (ncn_count_samples: no per-step copies in the timed region)
        count_acc = torch.zeros(2, dtype=torch.float64, device=dev)
        trainer.render_kwargs["count_acc"] = count_acc
        distill = None
        if state == "refreshed":
            fx = (synthetic.IMG_W / 2) / math.tan(synthetic.HFOV / 2)
            K = torch.tensor([[fx, 0, synthetic.IMG_W / 2], [0, fx, synthetic.IMG_H / 2], [0, 0, 1]])
            model.mark_invisible_cells(K, dev, torch.from_numpy(scene.poses).to(dev),
                                       (synthetic.IMG_W, synthetic.IMG_H), 0.01)
        else:
            with torch.no_grad():
                model.density_grid.copy_(torch.from_numpy(scene.density_grid).to(dev) * 10.0)
                model.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
            if state == "opaque":  # converged opaque surfaces (distill_opaque), then the same timed steps
                distill = distill_opaque(model, trainer, scene, dev)
        if pretrain > 0:  # a pool of 64 batches
            pool = [scene.torch_batch(args.rays, seed=rank * 10007 + 1000 + i, device=dev, gt=GT) for i in range(64)]
            trainer.update_grid = state == "refreshed"
            for k in range(pretrain):
                trainer.step(pool[k % len(pool)], global_step=k)
            trainer.update_grid = not args.no_grid_update
            torch.cuda.synchronize()
            del pool
        n_batches = 8
        batches = [scene.torch_batch(args.rays, seed=rank * 10007 + i, device=dev, gt=GT) for i in range(n_batches)]
        # past the clustering ramp (losses.py:217): full 2e-3 weights; refresh phase as window_start
        step0, n_refresh = window_start(max(3000, pretrain), args.warmup, steps)
        if args.no_grid_update:
            n_refresh = 0
        if trainer.update_grid and state != "refreshed":  # first-call costs of the refresh path stay out of the timed region
            model.update_density_grid(0.01 * 1024 / 3 ** 0.5, warmup=False)
        for k in range(args.warmup):
            trainer.step(batches[k % n_batches], global_step=step0 + k)
        trainer.flush_optimizer()  # (the timed region holds exactly `steps` optimizer steps)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        count_acc.zero_()
        if args.no_graph and kernel_table:
            _lib.TIMING = {n: [] for n in TIMED}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            trainer.step(batches[(args.warmup + k) % n_batches], global_step=step0 + args.warmup + k)
        trainer.flush_optimizer()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        tot = count_acc.clone()
        if not args.no_graph and kernel_table:
            # Per-kernel durations (the `kernels` table): a graph replay has no host launch to bracket,
            # so the captured body is run eagerly for `steps` more steps with HIP events on the launch
            # stream around each hot kernel (GPU spin in front: see _lib.TIMING).
            _lib.TIMING = {n: [] for n in TIMED}
            step_t = torch.full((), step0, dtype=torch.int64, device=dev)
            for k in range(steps):
                trainer._body(batches[k % n_batches], step_t, trainer._with_opt)
                if not trainer._with_opt:
                    trainer.opt.step(grad_scale=distributed.reduce_gradients(model))
            torch.cuda.synchronize()
        timing = _lib.TIMING or {}
        _lib.TIMING = None
        elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
        rank_ms = [round(1e3 * (t1 - t0) / steps, 3)]
        if world > 1:
            gathered = [torch.zeros_like(elapsed) for _ in range(world)]
            dist.all_gather(gathered, elapsed)
            rank_ms = [round(1e3 * float(g.item()) / steps, 3) for g in gathered]
            dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
            dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        return dict(el=float(elapsed.item()), tot=tot, rank_ms=rank_ms, timing=timing, model=model, batches=batches,
                    distill=distill, n_refresh=n_refresh)

    main_run = measure(args.precision, args.steps, True, args.pretrain)
    el, tot, rank_ms, timing = main_run["el"], main_run["tot"], main_run["rank_ms"], main_run["timing"]
    model, batches = main_run["model"], main_run["batches"]
    n_refresh = main_run["n_refresh"]
    kern = {}
    for name, evs in timing.items():
        if evs:
            ms = [a.elapsed_time(b) for a, b in evs]
            kern[name] = {"avg_us": round(1e3 * float(np.mean(ms)), 2), "launches": len(ms)}
    log(f"main run: {args.rays * world * args.steps / el:.1f} rays/s; roofline launches")
    cf_bytes_per_launch, cf_t = composite_fw_roofline(model, batches, dev, SyntheticScene())
    cf_us = cf_t["hbm"]
    traffic, traffic_src = pmc_traffic()
    del main_run, model, batches
    second = None
    if not args.no_bf16_line:  # the same step with the other MLP operand type (configs[2] asks for bf16)
        prec2 = "bf16" if args.precision == "fp16" else "fp16"
        r2 = measure(prec2, args.steps, False, args.pretrain)
        second = {"precision": prec2, "value": round(args.rays * world * args.steps / r2["el"], 1), "unit": "rays/s",
                  "ms_per_step": round(1e3 * r2["el"] / args.steps, 3),
                  "samples_per_s": round(float(r2["tot"][0].item()) / r2["el"], 1),
                  "workload": "configs[2]: the same full training step (normal clustering on), " + prec2 +
                              "-operand MFMA in the field MLP"}
        del r2
    extra = {}
    if not args.no_extra_states:
        for key, pre, st, what in (
                ("init_state", 0, "procedural", "random-init NGPMT on the procedural occupancy grid: rays never "
                                                "terminate early"),
                ("pretrained_state", 500, "procedural",
                 "NGPMT trained 500 untimed steps on the procedural occupancy grid (not refreshed meanwhile), then "
                 "the same timed steps; the refreshes in the timed steps re-grow the grid from the trained model's "
                 "densities.  No ray terminates early in this state (vr_samples_per_ray == rm_samples_per_ray: the "
                 "photometric + opacity losses keep T well above 1e-4 on this room for thousands of steps, "
                 "tools/trained_state_probe.py)"),
                ("opaque_state", 0, "opaque",
                 "converged opaque surfaces: the field's density fitted to the procedural room's occupancy "
                 "(bench.distill_opaque: 300 untimed Adam steps on log sigma, sigma 3000 inside occupied voxels), then "
                 "the same timed training steps: rays terminate at the first surface (vr_samples_per_ray << "
                 "rm_samples_per_ray), the compositors' early-stop paths on every ray"),
                ("refreshed_state", 500, "refreshed",
                 "the occupancy grid train_nerf.py maintains itself: mark_invisible_cells, then refreshed from the "
                 "model every 16 steps from step 0 (all cells for 256 steps) over 500 training steps; this "
                 "synthetic room's grid is then far denser than the procedural one (more samples per ray)")):
            if pre == args.pretrain and st == "procedural":
                continue  # (the headline measurement)
            r3 = measure(args.precision, args.steps, False, pre, st)
            if key == "opaque_state" and world == 1 and not args.no_eval_render:
                log("eval_render")
                extra["eval_render"] = dict(eval_render(r3["model"], SyntheticScene(), dev),
                                            model="the opaque_state model (converged opaque surfaces)")
            n_r = args.rays * world * args.steps
            extra[key] = {"value": round(n_r / r3["el"], 1), "unit": "rays/s",
                          "ms_per_step": round(1e3 * r3["el"] / args.steps, 3),
                          "samples_per_s": round(float(r3["tot"][0].item()) / r3["el"], 1),
                          "vr_samples_per_s": round(float(r3["tot"][1].item()) / r3["el"], 1),
                          "rm_samples_per_ray": round(float(r3["tot"][0].item()) / n_r, 2),
                          "vr_samples_per_ray": round(float(r3["tot"][1].item()) / n_r, 2),
                          "pretrain_steps": pre, "state": what}
            if r3.get("distill") is not None:
                extra[key]["distill_loss"] = r3["distill"]
            del r3
        # config #5's preset (ScanNet-Manhattan hyper-parameters: cluster weights 1e-2) on the same inputs
        r5 = measure(args.precision, args.steps, False, args.pretrain, "procedural", "scannet_manhattan")
        extra["other_config"] = {"preset": "scannet_manhattan", "value": round(args.rays * world * args.steps / r5["el"], 1),
                                 "unit": "rays/s", "ms_per_step": round(1e3 * r5["el"] / args.steps, 3),
                                 "workload": "configs[4]'s hyper-parameters (experiments/scannet_man/hyperparameters.py:"
                                             " loss_norm_D_C_* = 1e-2) on the synthetic Hypersim-shaped inputs"}
        del r5
    achieved = cf_bytes_per_launch / (cf_us * 1e-6) / 1e9
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    rays_total = args.rays * world * args.steps
    value = rays_total / el
    out = {
        "metric": "training rays/sec (+ samples/sec)",
        "value": round(value, 1),
        "unit": "rays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * el / args.steps, 3),
        "world": world,
        "backend": backend,
        "rank_ms_per_step": rank_ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": f"fp32 (march/composite/losses); {args.precision}-operand MFMA with fp32 accumulate in the field MLP",
        "data": "synthetic Hypersim-shaped batches (ai_001_001 box, 8x8 patches, procedural room, "
                "surface_bright target colours); " + (
                    f"NGPMT pretrained {args.pretrain} untimed steps from random init on the procedural occupancy "
                    f"grid" if args.pretrain > 0 else
                    "random-init NGPMT on the procedural occupancy grid (other states: pretrained_state, "
                    "opaque_state, refreshed_state)"),
        "config": {"workload": "configs[1]+[2]: full training step, 8192 rays/GPU, normal clustering on",
                   "rays_per_gpu": args.rays, "global_batch": args.rays * world, "grid": 128, "max_samples": 1024,
                   "parallelism": f"dp{world}", "grid_update_every_16": not args.no_grid_update,
                   "grid_refreshes_timed": n_refresh,
                   "grad_wire": ("fp16(fp16(S*g)/world): the reference's DDP wire, divided by the world before "
                                 "the SUM as DDP's default hook; optimizer grad_scale 1" if args.precision == "fp16" and
                                 distributed.DP_WIRE != "fp32" else "fp32 (SUM, 1/world in the optimizer)")
                   if world > 1 else None,
                   "step": "eager" if args.no_graph else "hip_graph" + (
                       "" if args.no_defer else " (optimizer of step k beside the marcher of step k+1)") + (
                       "" if args.no_split else " (photometric backward beside the normal clustering)")},
        "samples_per_s": round(float(tot[0].item()) / el, 1),
        "vr_samples_per_s": round(float(tot[1].item()) / el, 1),
        "rm_samples_per_ray": round(float(tot[0].item()) / rays_total, 2),
        "vr_samples_per_ray": round(float(tot[1].item()) / rays_total, 2),
        "roofline": {"kernel": "composite_train_fw (ncn_composite_train_fw_bg, the step's compositor)",
                     "bound": "hbm", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "frac_of_measured_copy": round(achieved / HBM_COPY_GBS, 4),
                     "measured_copy_gbs": HBM_COPY_GBS,
                     "traffic": traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": round(cf_bytes_per_launch),
                     "avg_launch_us": round(cf_us, 2),
                     "warm_us": round(cf_t["warm"], 2),
                     "frac_warm": round(cf_t["warm_bytes"] / (cf_t["warm"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                     "in_step_us": round(cf_t["in_step"], 2),
                     "batch65536": {"avg_launch_us": round(cf_t["big_us"], 2),
                                    "algorithmic_bytes_per_launch": round(cf_t["big_bytes"]),
                                    "frac": round(cf_t["big_bytes"] / (cf_t["big_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                                    "method": "one launch over config #4's global batch (65536 rays), 12 launches "
                                              "cycling through 3 sets of ~140 MB (HBM-cold), HIP events around all"},
                     "single_launch_floor": {"us": 5.1, "frac": 0.41,
                                             "note": "a load-only kernel of the same grid over the same ~19 MB "
                                                     "(round 4, DESIGN section 7): the launch ramp plus one round "
                                                     "of loads at ~6.3 TB/s bound one 8192-ray launch at ~0.41 of "
                                                     "the 8 TB/s spec before any arithmetic"},
                     "method": "avg_launch_us (-> achieved, frac): 48 back-to-back launches cycling through 24 "
                               "input sets (~16.5 MB each, ~400 MB in all, ~1.5x the 256 MiB Infinity Cache, so "
                               "each set is evicted before it is read again), HIP events on the launch stream "
                               "around all of them behind a GPU spin; "
                               "warm_us: the same on one set (cache-resident); in_step_us: one launch right behind "
                               "the field forward that produced its inputs, its own event pair (launch ramp and "
                               "event overhead included). Algorithmic bytes 24*S_vr + 4*S + 52*R (SURVEY 8d)"},
        "kernels": kern,
    }
    if second is not None:
        out["other_precision"] = second
    out.update(extra)
    if world == 1 and not args.no_cpu_baseline:
        log("cpu baseline")
        out["cpu_baseline"] = cpu_baseline()
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
