"""The host-built faiss k-means plan (ncn_kmeans_plan_fill, std::mt19937 in libncnerf.so's host code)
against the oracle's restatement of faiss's draws (oracle/losses_ref.py: rand_perm over a Python
mt19937, subsample_training_set, init picks, split_clusters' rand_float).  Runs on the CPU: the
plan builder is host code (no GPU call)."""
import numpy as np
import pytest
import torch

from oracle import losses_ref as L
from ncnerf_amd import _lib
from ncnerf_amd._lib import I32, U32, ptr


def test_mt19937_known_answer():
    """C++ [rand.predef]: the 10000th output of a default-constructed mt19937 (seed 5489) is 4123659995."""
    r = L.Mt19937(5489)
    for _ in range(9999):
        r()
    assert r() == 4123659995


def _plan(n_tri, K, seed=1234):
    lib = _lib.lib()
    words = int(lib.ncn_kmeans_plan_words(I32(n_tri), I32(K)))
    buf = torch.zeros(words, dtype=torch.int32)
    assert lib.ncn_kmeans_plan_fill(I32(n_tri), I32(K), U32(seed), ptr(buf)) == 0
    return buf.numpy().view(np.uint32)


@pytest.mark.parametrize("n_tri,K,rows", [(6272, 20, [20, 21, 57, 5120, 5121, 5800, 6272]), (3000, 10, [10, 11, 2560,
                                                                                                         2561, 3000])])
def test_plan_matches_oracle(n_tri, K, rows):
    p = _plan(n_tri, K)
    assert p[0] == 0x4B4D5031 and list(p[1:5]) == [n_tri, K, K * 256, L.N_RAND]
    init = p[p[5]:p[6]].view(np.uint16)
    cap, mw = K * 256, (n_tri + 31) // 32
    for nx in rows:
        sub, picks = L.faiss_training_set(nx, K)
        if nx == K:
            picks = np.arange(K)  # faiss's nx == k corner case copies the points in order
        assert np.array_equal(init[nx * K:(nx + 1) * K], picks), nx
        if nx > cap:
            row = p[p[6] + (nx - cap - 1) * mw:p[6] + (nx - cap) * mw]
            want = L.plan_mask_row(nx, K)
            assert np.array_equal(row[:len(want)], want) and not row[len(want):].any(), nx
            assert int(np.unpackbits(row.view(np.uint8)).sum()) == cap
    rnd = p[p[7]:p[7] + L.N_RAND].view(np.float32)
    assert np.array_equal(rnd, L.rand_floats(1234, L.N_RAND))


def test_oracle_kmeans_subsamples_above_cap():
    """faiss trains on K*256 points when given more; the final search still labels every point."""
    rng = np.random.default_rng(0)
    x = rng.normal(size=(6272, 3)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    C, a = L.spherical_kmeans(x, K=20, niter=20)
    assert C.shape == (20, 3) and a.shape == (6272,)
    np.testing.assert_allclose(np.linalg.norm(C, axis=1), 1.0, atol=1e-6)
    # the centroids are those of faiss's training subset: recompute one Lloyd update on it
    sub, _ = L.faiss_training_set(6272, 20)
    assert len(sub) == 5120 and len(set(sub.tolist())) == 5120
