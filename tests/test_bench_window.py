"""bench.py's timed window holds the long-run share of grid refreshes (Trainer.update_interval = 16,
train_nerf.py:318): round(K / 16) refreshes in K timed steps, whatever K and the warm-up."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


@pytest.mark.parametrize("steps", [1, 5, 8, 15, 16, 20, 24, 30, 32, 50, 100])
@pytest.mark.parametrize("warmup", [0, 3, 5])
def test_window_holds_round_share_of_refreshes(steps, warmup):
    base = 3000
    s0, n = bench.window_start(base, warmup, steps)
    assert base <= s0 < base + 16
    first = s0 + warmup
    refreshes = sum(1 for g in range(first, first + steps) if g % 16 == 0)
    assert refreshes == n == int(steps / 16 + 0.5)
