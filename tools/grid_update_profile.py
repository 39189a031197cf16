"""Time the occupancy-grid refresh (NGPMT.update_density_grid) piece by piece (diagnostic)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]
import torch
from ncnerf_amd import vren
from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers
from ncnerf_amd.synthetic import SyntheticScene

dev = torch.device("cuda:0")
scene = SyntheticScene()
m = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
m.density_grid.copy_(torch.from_numpy(scene.density_grid).to(dev) * 10)
thr = 0.01 * 1024 / 3 ** 0.5
for warm in (True, False, False, False):
    torch.cuda.synchronize(); t = time.perf_counter()
    m.update_density_grid(thr, warmup=warm)
    torch.cuda.synchronize(); print("update warmup=%s %.2f ms" % (warm, 1e3 * (time.perf_counter() - t)))
def T(name, f):
    torch.cuda.synchronize(); t = time.perf_counter(); r = f(); torch.cuda.synchronize()
    print("%-28s %.3f ms" % (name, 1e3 * (time.perf_counter() - t))); return r
cells = T("sample cells", lambda: m.sample_uniform_and_occupied_cells(128 ** 3 // 4, thr))
idx, coords = cells[0]
xyz = T("xyz", lambda: ((coords / 127 * 2 - 1) * (0.5 - 0.5 / 128)).contiguous())
T("density 1M", lambda: m.density(xyz))
T("density 1M again", lambda: m.density(xyz))
tmp = torch.zeros_like(m.density_grid)
T("scatter", lambda: tmp.__setitem__((0, idx), m.density(xyz)))
T("where", lambda: torch.where(m.density_grid < 0, m.density_grid, torch.maximum(m.density_grid * 0.95, tmp)))
T("mean item", lambda: m.density_grid[m.density_grid > 0].mean().item())
T("packbits", lambda: vren.packbits(m.density_grid, 1.0, m.density_bitfield))
T("nonzero", lambda: torch.nonzero(m.density_grid[0] > thr))
