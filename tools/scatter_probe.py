"""Diagnostic: time ncn_field_scatter alone (and diagnostic builds of it) on realistic marched
samples: the bench batch is marched, the field run forward and the MLP backward pass once, then
the scatter is timed per library (main + tools/_build/field_*.so).  Not part of the product."""
import ctypes
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ncnerf_amd import _lib  # noqa: E402
from ncnerf_amd._lib import F32, I32, I64, ptr, stream  # noqa: E402
from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers  # noqa: E402
from ncnerf_amd.rendering import march_train_fused  # noqa: E402
from ncnerf_amd.synthetic import SyntheticScene  # noqa: E402

dev = torch.device("cuda:0")
scene = SyntheticScene()
model = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
model.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
b = scene.torch_batch(8192, seed=1, device=dev)
o, d = b["rays_o"].contiguous(), b["rays_d"].contiguous()
mk = march_train_fused(model, o, d, 0.01, 1024, noise=torch.rand(8192, device=dev))
n = int(mk["counter"][0].item())
xyzs, dirs = mk["xyzs"][:n].contiguous(), mk["dirs"][:n].contiguous()
print("samples", n, flush=True)
main = _lib.lib()
packed = model._pack_weights()
enc = torch.empty(((n + 15) // 16) * 64 * 8, dtype=torch.float16, device=dev)
sig = torch.empty(n, device=dev)
rgb = torch.empty(n, 3, device=dev)
table = model.flat_params()[: model._n_table]
gen = torch.Generator(device="cuda").manual_seed(0)
dsig = torch.randn(n, device=dev, generator=gen) * 1e-3
drgb = torch.randn(n, 3, device=dev, generator=gen) * 1e-3
nb = main.ncn_field_bwd_blocks(I64(n))
slab = torch.empty(nb * 19712, device=dev)
dE = torch.empty(int(main.ncn_field_bwd_dE_floats(I64(n))), device=dev)
lmax = torch.empty(16 * 256, device=dev)
gtab = torch.zeros_like(table)
order = torch.empty(n, dtype=torch.int32, device=dev)
ORDER = [None]


def ev_time(f, reps=20):
    f()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, e in evs:
        torch.cuda._sleep(100000)
        a.record()
        assert f() == 0
        e.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(e) for a, e in evs]) * 1e3)


def prepare(sorted_):
    """fwd + MLP backward in the chosen processing order (dE in that order)."""
    ORDER[0] = order if sorted_ else None
    o = ORDER[0]
    srt = lambda: main.ncn_field_sort_windows(ptr(xyzs), I64(n), ptr(None), F32(model._xyz_min),  # noqa: E731
                                              F32(model._xyz_extent), ptr(order), stream())
    if sorted_:
        print(f"  sort_windows {ev_time(srt):7.1f} us", flush=True)
    fwd = lambda: main.ncn_field_fwd(ptr(xyzs), ptr(dirs), I64(n), ptr(None), ptr(o), ptr(table),  # noqa: E731
                                     model._levels_ptr, F32(model._xyz_min), F32(model._xyz_extent), ptr(packed),
                                     I32(0), I32(0), ptr(sig), ptr(rgb), ptr(enc), stream())
    mlp = lambda: main.ncn_field_bwd_mlp(ptr(xyzs), ptr(dirs), I64(n), ptr(None), ptr(o), ptr(packed), I32(0), ptr(enc),  # noqa: E731
                                         ptr(dsig), ptr(drgb), ptr(None), ptr(slab), ptr(dE), ptr(lmax), stream())
    print(f"  field_fwd {ev_time(fwd):7.1f} us   bwd_mlp {ev_time(mlp):7.1f} us", flush=True)
    return sig.clone(), rgb.clone()


def scat(lib, lo=0, hi=16):
    return lib.ncn_field_scatter(ptr(xyzs), I64(n), ptr(None), ptr(ORDER[0]), model._levels_ptr, F32(model._xyz_min),
                                 F32(model._xyz_extent), ptr(dE), ptr(lmax), I32(lo), I32(hi), I32(0), ptr(gtab),
                                 stream())


def timeit(lib, reps=20, **kw):
    return ev_time(lambda: scat(lib, **kw), reps)


libs = [("main", main)]
for so in [] if os.environ.get("SCATTER_PROBE_MAIN_ONLY") else sorted(glob.glob(os.path.join(ROOT, "tools", "_build", "field_*.so"))):
    L = ctypes.CDLL(so)
    L.ncn_field_scatter.argtypes = _lib.SIGNATURES["ncn_field_scatter"]
    L.ncn_field_scatter.restype = ctypes.c_int
    L.ncn_field_fwd.argtypes = _lib.SIGNATURES["ncn_field_fwd"]
    L.ncn_field_fwd.restype = ctypes.c_int
    libs.append((os.path.basename(so)[6:-3], L))
gref = None
for sorted_ in (False,) if os.environ.get("SCATTER_PROBE_MAIN_ONLY") or os.environ.get("SCATTER_PROBE_IDENTITY") else (False, True):
    print("order:", "Morton windows" if sorted_ else "ray (identity)", flush=True)
    so = prepare(sorted_)
    if sorted_:
        print(f"  fwd outputs vs identity order: max|dsigma| {float((so[0] - s0[0]).abs().max()):.3e} "
              f"max|drgb| {float((so[1] - s0[1]).abs().max()):.3e}")
    else:
        s0 = so
    for name, L in libs:
        # each library's own MLP pass first: it writes the positions in that library's unit layout
        L.ncn_field_bwd_mlp.argtypes = _lib.SIGNATURES["ncn_field_bwd_mlp"]
        L.ncn_field_bwd_mlp.restype = ctypes.c_int
        assert L.ncn_field_bwd_mlp(ptr(xyzs), ptr(dirs), I64(n), ptr(None), ptr(ORDER[0]), ptr(packed), I32(0), ptr(enc),
                                   ptr(dsig), ptr(drgb), ptr(None), ptr(slab), ptr(dE), ptr(lmax), stream()) == 0
        gtab.zero_()
        assert scat(L) == 0
        torch.cuda.synchronize()
        g1 = gtab.clone()
        msg = ""
        if gref is None:
            gref = g1
        else:
            rel = ((g1 - gref).norm() / gref.norm()).item()
            msg = f"rel-L2 vs first {rel:.2e}"
        if os.environ.get("SCATTER_PROBE_FWD"):  # (the forward of each library, same inputs)
            fw = lambda: L.ncn_field_fwd(ptr(xyzs), ptr(dirs), I64(n), ptr(None), ptr(ORDER[0]), ptr(table),  # noqa: E731
                                         model._levels_ptr, F32(model._xyz_min), F32(model._xyz_extent), ptr(packed),
                                         I32(0), I32(0), ptr(sig), ptr(rgb), ptr(enc), stream())
            t_fw = ev_time(fw)
            out = (sig.clone(), rgb.clone(), enc.clone())
            if name == "main":
                FWD_REF = out
            same = all(torch.equal(a, b) for a, b in zip(out, FWD_REF))
            print(f"  {name:24s} field_fwd {t_fw:7.1f} us  bit-identical to main: {same}", flush=True)
            continue
        t = timeit(L)
        coarse = timeit(L, lo=0, hi=10)
        fine = timeit(L, lo=10, hi=16)
        print(f"  {name:24s} all {t:7.1f} us  levels0-9 {coarse:7.1f}  levels10-15 {fine:7.1f}  {msg}", flush=True)
        if os.environ.get("SCATTER_PROBE_PER_LEVEL"):
            print("   per level:", " ".join(f"{l}:{timeit(L, lo=l, hi=l + 1):.1f}" for l in range(16)), flush=True)
        if hasattr(L, "ncn_diag_sc_span"):  # per-workgroup start/end (100 MHz realtime) and shader cycles
            assert scat(L) == 0
            torch.cuda.synchronize()
            buf = (ctypes.c_ulonglong * (256 * 20))()
            L.ncn_diag_sc_span(buf)
            a = np.frombuffer(buf, dtype=np.uint64).reshape(256, 20).astype(np.float64)
            os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
            np.save(os.path.join(ROOT, "gpurun_out", f"sc_span_{name}.npy"), a)
            # per-unit durations (us) by level, and a greedy dynamic assignment of the same units in
            # the same order (each to the earliest-free workgroup) with those durations
            spans = [32768 if l < 6 else 16384 if l < 10 else 4096 if l < 15 else 2048 for l in range(16)]
            lev = np.concatenate([np.full(-(-n // sp), l) for l, sp in enumerate(spans)])
            dur = {}
            for b in range(256):
                prev = a[b, 0]
                for k in range(8):
                    if a[b, 5 + 2 * k] == 0:
                        break
                    u = int(a[b, 4 + 2 * k])
                    dur[u] = (a[b, 5 + 2 * k] - prev) / 100.0
                    prev = a[b, 5 + 2 * k]
            byl = {}
            for u, d in dur.items():  # (a variant with other unit spans: levels past the default table as -1)
                byl.setdefault(int(lev[u]) if u < len(lev) else -1, []).append(d)
            print("     unit us by level (median):", " ".join(f"{l}:{np.median(v):.1f}" for l, v in sorted(byl.items())))
            free = np.zeros(256)
            for u in sorted(dur):
                i = int(np.argmin(free))
                free[i] += dur[u]
            print(f"     greedy dynamic makespan with these durations: {free.max():.1f} us (static: {(a[:, 1] - a[:, 0]).max() / 100:.1f})")
            t0 = a[:, 0].min()
            st, en = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0  # us
            ghz = np.median((a[:, 3] - a[:, 2]) / ((a[:, 1] - a[:, 0]) * 10.0))
            pq = lambda v: " ".join(f"{x:.1f}" for x in np.percentile(v, [0, 10, 50, 90, 100]))  # noqa: E731
            print(f"     WG span (us; min p10 p50 p90 max): start {pq(st)}  end {pq(en)}  busy {pq(en - st)}  "
                  f"shader clock {ghz:.2f} GHz", flush=True)
        if hasattr(L, "ncn_diag_sc_times"):
            buf = (ctypes.c_ulonglong * (256 * 10))()
            L.ncn_diag_sc_times(buf, 1)
            assert scat(L) == 0
            torch.cuda.synchronize()
            L.ncn_diag_sc_times(buf, 0)
            a = np.frombuffer(buf, dtype=np.uint64).reshape(256, 10).astype(np.float64)
            names = ["load", "work", "drain", "barrier", "flush"]
            print("     cycles per WG (wave 0, mean), coarse | fine:",
                  "  ".join(f"{nm} {a[:, 2 * i].mean():.0f}|{a[:, 2 * i + 1].mean():.0f}" for i, nm in enumerate(names)))
            tot = a.sum(1) - a[:, 4]  # (the coarse drains are inside the coarse work)
            q = np.percentile(tot, [0, 10, 50, 90, 100])
            print("     total cycles per WG: min %.0f p10 %.0f median %.0f p90 %.0f max %.0f" % tuple(q))
