"""CPU check of the closed-form chain behind the wave-parallel marcher (csrc/vren.hip march_chain).

The reference walk advances t by repeated float32 adds c_{k+1} = fl(c_k + dt) (raymarching.cu:221-233).
march_chain computes a window of that chain in closed form (constant bit-pattern step inside a binade,
real adds for the first two steps of a binade and for the step that leaves it).  This transcribes the
same algorithm with numpy float32/uint32 and compares it against the serial adds over many starting
points and step sizes, including the one binade where dt/ulp is a tie (round-half-even) and t = 0.
"""
import numpy as np
import pytest

F = np.float32


def _bits(x):
    return int(np.array(x, dtype=np.float32).view(np.uint32))


def _flt(b):
    return F(np.array(b & 0xFFFFFFFF, dtype=np.uint32).view(np.float32))


def chain_closed_form(cb, dt, L):
    """Transcription of march_chain: returns c_0 .. c_L (L + 1 values)."""
    cb, dt = F(cb), F(dt)
    c = [None] * (L + 1)
    c[0] = cb
    j0, v = 0, cb
    while True:
        bv = _bits(v)
        v1 = F(v + dt)
        b1 = _bits(v1)
        r1, r = (b1 - bv) & 0xFFFFFFFF, 0
        if (bv >> 23) != (b1 >> 23) or bv == 0:
            K, vn = 0, v1
        else:
            v2 = F(v1 + dt)
            b2 = _bits(v2)
            if (b2 >> 23) != (b1 >> 23):
                K, vn = 1, v2
            else:
                r = b2 - b1
                assert r > 0
                top = bv | 0x7FFFFF
                kmax = (top - bv - r1) // r + 1
                K = min(kmax, L)
                vn = F(_flt(bv + r1 + (K - 1) * r) + dt)
        for i in range(j0 + 1, min(j0 + K, L) + 1):
            c[i] = _flt(bv + r1 + (i - j0 - 1) * r)
        if j0 + K >= L:
            return c
        J = j0 + K + 1
        c[J] = vn
        if J == L:
            return c
        j0, v = J, vn


def chain_serial(cb, dt, L):
    out = [F(cb)]
    for _ in range(L):
        out.append(F(out[-1] + F(dt)))
    return out


def _check(cb, dt, L=128):
    a = np.array(chain_closed_form(cb, dt, L), dtype=np.float32)
    b = np.array(chain_serial(cb, dt, L), dtype=np.float32)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (cb, dt, np.argwhere(a != b)[:3])


def test_chain_config_dt():
    dt = F(F(1.73205080757) / F(1024))  # sqrt(3)/max_samples, the configs' constant step
    rng = np.random.default_rng(0)
    starts = [0.0, 0.01, F(0.01) + dt * F(0.37), 1e-6, 0.0155, 0.0156249, 0.5 - 1e-7, 0.999, 1.9999]
    starts += list(rng.uniform(0.0, 2.0, 300)) + list(rng.uniform(0.0, 0.05, 300))
    for cb in starts:
        _check(F(cb), dt, 128)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_chain_random_dt(seed):
    rng = np.random.default_rng(seed)
    for _ in range(150):
        dt = F(rng.uniform(1e-4, 2e-2))
        cb = F(rng.uniform(0.0, 1.5))
        _check(cb, dt, 192)


def test_chain_tie_binade():
    # dt with few mantissa bits: dt/ulp is an exact half-integer in one binade -> round-half-even
    for dt in (F(2 ** -10 * 1.5), F(2 ** -9 * 1.25), F(3 * 2 ** -12), F(0.001953125)):
        for cb in (0.0, F(dt) * F(1.5), F(2 ** -8), F(2 ** -8) + F(2 ** -31), F(0.0041), F(0.3)):
            _check(F(cb), dt, 256)
