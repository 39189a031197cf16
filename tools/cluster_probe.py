"""Diagnostic (not product): phase timestamps of the one-launch clustering kernel (a
tools/build_loss_variants.sh NCN_DIAG_CL_TIMES build) on 6272 Manhattan-like normals."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ncnerf_amd import _lib  # noqa: E402

so = os.environ.get("NCN_CL_PROBE_SO", os.path.join(ROOT, "tools", "_build", "lib_ncn_diag_cl_times.so"))
_lib.LIB_PATH = so
L = _lib.lib()
from ncnerf_amd import losses as Lo  # noqa: E402

dev = torch.device("cuda:0")
rng = np.random.default_rng(0)
axes = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], np.float32)
x = axes[rng.choice(6, 6272)] + rng.normal(0, 0.05, (6272, 3)).astype(np.float32)
x /= np.linalg.norm(x, axis=1, keepdims=True)
n = torch.from_numpy(x.astype(np.float32)).to(dev)
for _ in range(5):
    Lo.cluster_losses(n)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 64)()
L.ncn_diag_cl_times(buf)
t = np.array(buf[:], dtype=np.float64)
t0 = t[0]
print("compaction", (t[1] - t0) / 100.0, "us (100 MHz ticks)")
for it in range(21):
    a, b, c = t[2 + 2 * it], t[3 + 2 * it], t[2 + 2 * (it + 1)] if it < 20 else t[60]
    print(f"it {it:2d}: start {(a - t0) / 100:7.2f}  compute {(b - a) / 100:6.2f}  to-next {(c - b) / 100:6.2f}")
print("total", (t[60] - t0) / 100.0)
names = {56: "compaction pass 1 + scan", 57: "after final barrier (cnt ready)", 58: "select done",
         59: "p2 barrier passed", 61: "stats done", 62: "p3 barrier passed", 63: "st3 read", 60: "end"}
for k in sorted(names):
    print(f"{names[k]:32s} {(t[k] - t0) / 100:8.2f}")
