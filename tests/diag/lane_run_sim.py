"""Diagnostic (CPU): what merging runs ACROSS lanes would save the fine-level table scatter
(DESIGN §7 "Next", item 1).

The product's fine units hand a wave 64 x 2-sample grabs (lane i: samples 2i, 2i + 1 of the grab)
and sum a lane's consecutive samples in one cell in registers (sc_direct), so one record (8 corners'
LDS adds) goes out per in-lane run.  Counted here on one marched 8192-ray bench batch (oracle
marcher), per fine level, records (= 8-corner add groups) per 128-sample grab:
* now: in-lane runs (a lane's 2 samples merge when they share a cell);
* cross-lane runs: the grab's 128 samples as one sequence, a run of equal cells continued over the
  lane boundary (what a wave-wide segmented sum of adjacent lanes would leave);
* distinct cells per grab (a full in-wave key match of cells);
* and the corner adds per grab against the distinct entries (a full in-wave match of entries, the
  VERDICT's estimate)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normal-clustering-nerf_amd")]
from oracle import field_ref, vren_ref  # noqa: E402
from ncnerf_amd.synthetic import SyntheticScene  # noqa: E402


def main():
    scene = SyntheticScene()
    b = scene.batch(8192, seed=1)
    o, d = b["rays_o"], b["rays_d"]
    _, ht, _ = vren_ref.ray_aabb_intersect(o, d, np.zeros((1, 3), np.float32), np.full((1, 3), 0.5, np.float32), 1)
    ht = ht[:, 0].copy()
    near = (ht[:, 0] >= 0) & (ht[:, 0] < 0.01)
    ht[near, 0] = 0.01
    noise = np.random.default_rng(0).random(8192).astype(np.float32)
    _, xyzs, _, _, _, cnt = vren_ref.raymarching_train(o, d, ht, scene.bitfield, 1, 0.5, 0.0, noise, 128, 1024)
    S = int(cnt[0])
    G = S // 128
    x = xyzs[:G * 128] + 0.5
    print("samples", S, "grabs", G)
    levels, _ = field_ref.grid_levels(0.5)
    for l in range(10, 16):
        lv = levels[l]
        hashed = lv["res"] ** 3 > lv["params"]
        pos = (x.astype(np.float64) * lv["scale"] + 0.5).astype(np.float32)
        pg = np.floor(pos).astype(np.int64)
        key = (pg[:, 0] * 4096 + pg[:, 1]) * 4096 + pg[:, 2]
        k = key.reshape(G, 64, 2)
        now = 64 + int((k[:, :, 1] != k[:, :, 0]).sum()) / G
        seq = key.reshape(G, 128)
        cross = 1 + int((seq[:, 1:] != seq[:, :-1]).sum()) / G
        distinct = float(np.mean([len(np.unique(r)) for r in seq]))
        ents = []
        for c in range(8):
            p = pg + np.array([(c >> q) & 1 for q in range(3)])
            if hashed:
                e = (p[:, 0] ^ (p[:, 1] * 2654435761) ^ (p[:, 2] * 805459861)) & 0xFFFFFFFF
            else:
                e = p[:, 0] + lv["res"] * p[:, 1] + lv["res"] ** 2 * p[:, 2]
            ents.append(e % lv["params"])
        E = np.stack(ents, 1).reshape(G, 128 * 8)
        dent = float(np.mean([len(np.unique(r)) for r in E]))
        print(f"level {l} res {lv['res']}: records per grab now {now:.1f}, cross-lane runs {cross:.1f} "
              f"({1 - cross / now:.1%} fewer), distinct cells {distinct:.1f} ({1 - distinct / now:.1%} fewer); "
              f"corner adds now {8 * now:.0f} vs distinct entries {dent:.0f}")


if __name__ == "__main__":
    main()
