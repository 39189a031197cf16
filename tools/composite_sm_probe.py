"""Diagnostic: time the sample-major training compositor (ncn_composite_train_fw_sm) of the main
library and of tools/_build/vren_sm_*.so variants (tools/build_sm_variants.sh) against the
ray-major ncn_composite_train_fw_bg, on marched bench batches (warm: one set; cold: cycling through
24 sets > the Infinity Cache), and report how often a wave's last segment runs past its range plus
look-ahead (host analysis of the sample codes).  Not part of the product."""
import ctypes
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ncnerf_amd import _lib  # noqa: E402
from ncnerf_amd._lib import F32, I32, I64, P, ptr, stream  # noqa: E402
from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers  # noqa: E402
from ncnerf_amd.rendering import march_buffers, march_train_fused  # noqa: E402
from ncnerf_amd.synthetic import SyntheticScene  # noqa: E402

dev = torch.device("cuda:0")
scene = SyntheticScene()
model = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
model.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
sets = []
with torch.no_grad():
    for j in range(24):
        b = scene.torch_batch(8192, seed=j % 8, device=dev)
        mk = march_train_fused(model, b["rays_o"].contiguous(), b["rays_d"].contiguous(), 0.01, 1024,
                               noise=torch.rand(8192, device=dev), out=march_buffers(8192, 1024, dev, codes=True))
        S = int(mk["counter"][0].item())
        out = model(mk["xyzs"], mk["dirs"], n_samples_dev=mk["counter"])
        R = 8192
        k = {"sig": out["sigmas"][:S].clone(), "rgb": out["rgbs"][:S].clone(), "dl": mk["deltas"][:S].clone(),
             "ts": mk["ts"][:S].clone(), "ra": mk["rays_a"].clone(), "codes": mk["sample_ray"][:S].clone(), "S": S,
             "res": [torch.empty(R, dtype=torch.int64, device=dev), torch.empty(R, device=dev),
                     torch.empty(R, device=dev), torch.empty(R, 3, device=dev), torch.empty(S, device=dev),
                     torch.empty(R, 3, device=dev)]}
        sets.append(k)
        del out, mk

# host analysis of set 0: per 256-sample range, how far the owned last segment runs past the range
c = sets[0]["codes"].cpu().numpy()
S0 = c.shape[0]
starts = np.flatnonzero(np.concatenate([[True], c[1:] != c[:-1]]))
ends = np.concatenate([starts[1:], [S0]])
past = []
for base in range(0, S0, 256):
    e = base + 256
    # the segment containing sample e - 1, if it starts inside [base, e) and is short (> 0)
    i = np.searchsorted(starts, e - 1, side="right") - 1
    if starts[i] >= base and c[starts[i]] > 0 and ends[i] > e:
        past.append(ends[i] - e)
    else:
        past.append(0)
past = np.array(past)
lens = ends - starts
stats = {"S": S0, "ranges": len(past), "frac_past_0": float(np.mean(past > 0)), "frac_past_64": float(np.mean(past > 64)),
         "frac_past_128": float(np.mean(past > 128)), "max_past": int(past.max()),
         "long_rays": int(np.sum((c[starts] < 0))), "mean_seg": float(lens.mean())}
print(json.dumps(stats), flush=True)


def sm_args(k):
    R = k["ra"].shape[0]
    return [ptr(k["sig"]), ptr(k["rgb"]), ptr(k["dl"]), ptr(k["ts"]), ptr(k["codes"]), ptr(k["ra"]), I64(R),
            I64(k["S"]), ptr(None), I64(k["S"]), I32(3), F32(1e-4)] + [ptr(t) for t in k["res"][:5]] + [
                F32(1.0), ptr(k["res"][5]), stream()]


def rm_args(k):
    R = k["ra"].shape[0]
    return [ptr(k["sig"]), ptr(k["rgb"]), ptr(k["dl"]), ptr(k["ts"]), ptr(k["ra"]), I64(R), I64(k["S"]), I32(3),
            F32(1e-4)] + [ptr(t) for t in k["res"][:5]] + [F32(1.0), ptr(k["res"][5]), stream()]


def b2b(f, arg_list, n=48):
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(2_000_000)
    a.record()
    for i in range(n):
        f(*arg_list[i % len(arg_list)])
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / n


def bind(path):
    L = ctypes.CDLL(path)
    f = L.ncn_composite_train_fw_sm
    f.argtypes = _lib.SIGNATURES["ncn_composite_train_fw_sm"]
    f.restype = ctypes.c_int
    return f


ref = None
res = {}
rm = _lib.lib().ncn_composite_train_fw_bg
for k in sets:
    rm(*rm_args(k))
res["ray_major"] = {"cold": b2b(rm, [rm_args(k) for k in sets]), "warm": b2b(rm, [rm_args(sets[0])])}
libs = [("main", _lib.LIB_PATH)] + [(os.path.basename(p)[8:-3], p)
                                     for p in sorted(glob.glob(os.path.join(ROOT, "tools", "_build", "vren_sm_*.so")))]
for name, path in libs:
    f = bind(path)
    for k in sets:
        assert f(*sm_args(k)) == 0
    torch.cuda.synchronize()
    outs = [t.clone() for t in sets[0]["res"]]
    same = ref is None or all(torch.equal(a, b) for a, b in zip(outs, ref))
    if ref is None:
        ref = outs
    res[name] = {"cold": b2b(f, [sm_args(k) for k in sets]), "warm": b2b(f, [sm_args(sets[0])]), "same_as_main": same}
    print(name, json.dumps(res[name]), flush=True)
print(json.dumps(res))
