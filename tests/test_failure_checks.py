"""CPU checks of the trained-state test's infrastructure: the
failure dump writes the failing state and re-raises, and the kink-branch check passes branches that
flip within rounding distance of the kink and fails one flipped far from it."""
import json
import os

import numpy as np
import pytest

from failure_dump import dump_on_failure
from oracle import losses_ref
from kink_check import KINK_ABS, check_kink_flips, kink_flips
from test_oracle_kinks import _clustered_normals


def test_dump_written_on_failure_only(tmp_path):
    arrays = {"params": np.arange(10, dtype=np.float32), "noise": np.ones(4, np.float32), "none": None}
    with dump_on_failure("ok_case", arrays, {"step": 1}, base=str(tmp_path)):
        assert 1 + 1 == 2
    assert not os.path.exists(tmp_path / "ok_case")
    with pytest.raises(AssertionError) as ei:
        with dump_on_failure("bad_case", lambda: arrays, lambda: {"step": 3000, "v": np.float64(0.5)},
                             base=str(tmp_path)):
            assert 1 == 2, "forced"
    d = tmp_path / "bad_case"
    assert str(d) in str(ei.value) and "forced" in str(ei.value)
    z = np.load(d / "arrays.npz")
    assert sorted(z.files) == ["noise", "params"]
    np.testing.assert_array_equal(z["params"], arrays["params"])
    rec = json.load(open(d / "record.json"))
    assert rec["step"] == 3000 and rec["v"] == 0.5 and "forced" in rec["failure"]


def _perturbed(x, eps, seed):
    y = x + eps * np.random.default_rng(seed).standard_normal(x.shape).astype(np.float32)
    return (y / np.linalg.norm(y, axis=1, keepdims=True)).astype(np.float32)


def test_kink_flips_within_rounding_distance_pass():
    x, labels = _clustered_normals(1)
    y = _perturbed(x, 5e-4, 2)  # the two sides' normals ~5e-4 apart, as measured
    flips = kink_flips(y, x, labels)
    assert len(flips) > 0  # some L1 components sit within 5e-4 of their centroid
    check_kink_flips(flips)
    assert max(f["v_o"] for f in flips) <= 2e-3


def test_kink_flip_far_from_the_kink_fails():
    x, labels = _clustered_normals(1)
    y = x.copy()
    # a HIP-side normal whose component sits on the other branch, far from the kink
    _, vo_l1, _ = losses_ref.kink_values(x, labels)
    keep = np.flatnonzero(np.abs(labels) == 1)
    r, c = np.argwhere(np.abs(vo_l1[0]) > 2 * KINK_ABS)[0]
    i = keep[r]
    y[i, c] -= 2.0 * np.sign(labels[i]) * vo_l1[0][r, c]  # flips the sign of (n - c) there
    y[i] /= np.linalg.norm(y[i])
    flips = kink_flips(y, x, labels)
    assert any(f["v_o"] > KINK_ABS for f in flips)
    with pytest.raises(AssertionError, match="away from the kink"):
        check_kink_flips(flips)
