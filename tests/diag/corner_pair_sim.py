"""Diagnostic (CPU): what corner-pair slots would save the fine-level table scatter (DESIGN §7,
round-5 findings).

On hashed levels tcnn's index is (x ^ y*p1 ^ z*p2) mod T with p0 = 1, so for an even x the corners
x and x + 1 of one (y, z) edge hash to entries e and e ^ 1 — one 16-B pair.  A slot keyed by the
pair (e >> 1) could take both corners with ONE set lookup.  Counted on one marched 8192-ray bench
batch (oracle marcher), per fine level, with the product's units (4096 samples; 2048 on level 15):
* set lookups per sample now (8) and with pairs (4 per even x, 8 per odd x);
* distinct slots per unit (claims): entries now, pairs with pair slots;
* the share of wave-instructions in which all 64 lanes have an even x (only there would the
  second lookup of an edge be skipped for the whole wave; lanes of one instruction hold samples
  64 positions apart, as the product's grabs lay them out)."""
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
    x = xyzs[:S] + 0.5
    print("samples", S)
    levels, _ = field_ref.grid_levels(0.5)
    tot_now = tot_pair = 0
    for l in range(10, 16):
        lv = levels[l]
        hashed = lv["res"] ** 3 > lv["params"]
        pos = (x.astype(np.float64) * lv["scale"] + 0.5).astype(np.float32)
        pg = np.floor(pos).astype(np.int64)
        ents = []
        for c in range(8):
            p = pg + np.array([(c >> k) & 1 for k in range(3)])
            if hashed:
                e = (p[:, 0] ^ (p[:, 1] * 2654435761) ^ (p[:, 2] * 805459861)) & 0xFFFFFFFF
            else:
                e = p[:, 0] + lv["res"] * p[:, 1] + lv["res"] ** 2 * p[:, 2]
            ents.append(e % lv["params"])
        E = np.stack(ents, 1)
        even = (pg[:, 0] & 1) == 0
        # (mod T keeps e ^ 1 paired only when T is even — true for every level here)
        look_now = 8 * S
        look_pair = int(np.where(even, 4, 8).sum())
        unit = 2048 if l == 15 else 4096
        claims_now = claims_pair = 0
        for s in range(0, S, unit):
            blk = E[s:s + unit]
            claims_now += len(np.unique(blk))
            claims_pair += len(np.unique(blk >> 1))
        # wave-instructions: 64 lanes holding samples 64 apart inside a unit
        all_even = n_instr = 0
        for s in range(0, S - unit + 1, unit):
            ev = even[s:s + unit].reshape(64, -1)  # [lane][k]: sample s + lane * (unit / 64) + k
            all_even += int(ev.all(axis=0).sum())
            n_instr += ev.shape[1]
        tot_now += look_now
        tot_pair += look_pair
        print(f"level {l} res {lv['res']} hashed {hashed}: lookups/sample {look_now / S:.2f} -> {look_pair / S:.2f} "
              f"({1 - look_pair / look_now:.1%} fewer); claims/unit-sample {claims_now / S:.3f} -> {claims_pair / S:.3f}; "
              f"wave-instructions with all lanes even {all_even}/{n_instr}")
    print(f"levels 10-15: set lookups {tot_now} -> {tot_pair} ({1 - tot_pair / tot_now:.1%} fewer)")


if __name__ == "__main__":
    main()
