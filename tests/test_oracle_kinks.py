"""The oracle's shared-branch evaluation of the cluster terms (losses_ref.cluster_losses `signs`,
used by tests/test_gpu_trained_state.py): with the branches of the same normals it is the plain
evaluation — value and gradient — and with another evaluation's branches only the gradient of the
terms whose sign differs changes (and, through the centroid, their whole cluster's rows)."""
import numpy as np
import torch

from oracle import losses_ref


def _clustered_normals(seed, n=600, spread=0.02):
    rng = np.random.default_rng(seed)
    axes = np.eye(3)
    lab = rng.integers(1, 4, n)
    x = axes[lab - 1] + spread * rng.standard_normal((n, 3))
    flip = rng.random(n) < 0.3
    x[flip] *= -1
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    labels = np.where(flip, -lab, lab)
    labels[rng.random(n) < 0.1] = 0  # outside the selected clusters
    return x.astype(np.float32), labels


def _terms_and_grad(x, labels, signs=None):
    xt = torch.from_numpy(x).double().requires_grad_(True)
    ort, cdot, cl1 = losses_ref.cluster_losses(xt, torch.from_numpy(labels), signs=signs)
    (ort + cdot + cl1).backward()
    return [float(t) for t in (ort, cdot, cl1)], xt.grad.numpy().copy()


def test_own_branches_equal_plain_evaluation():
    x, labels = _clustered_normals(0)
    t0, g0 = _terms_and_grad(x, labels)
    t1, g1 = _terms_and_grad(x, labels, signs=losses_ref.kink_signs(x, labels))
    np.testing.assert_allclose(t1, t0, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(g1, g0, rtol=1e-12, atol=1e-15)


def test_other_branches_move_the_gradient_not_the_value():
    x, labels = _clustered_normals(1)
    y = x + 5e-4 * np.random.default_rng(2).standard_normal(x.shape).astype(np.float32)
    y /= np.linalg.norm(y, axis=1, keepdims=True)
    sx, sy = losses_ref.kink_signs(x, labels), losses_ref.kink_signs(y, labels)
    differ = int(sum((a != b).sum() for a, b in zip(sx[1], sy[1])))
    assert differ > 0  # some L1 components sit within 5e-4 of their centroid
    t_own, g_own = _terms_and_grad(y, labels)
    t_sh, g_sh = _terms_and_grad(y, labels, signs=sx)
    # value: |v| vs s*v differ only on the flipped branches, by 2|v| there (tiny)
    assert abs(t_sh[2] - t_own[2]) <= 2 * 5e-3 * differ / max(1, int((labels != 0).sum())) + 1e-12
    assert t_sh[1] == t_own[1]
    # gradient: the flipped branches' terms move it (through the centroid, every row of their cluster)
    assert not np.allclose(g_sh, g_own)
