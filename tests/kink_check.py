"""The kink-branch check of tests/test_gpu_trained_state.py: the
oracle evaluates |v| of the cluster terms (losses.py:461-478) on the HIP side's branches; every
branch it would have chosen otherwise must sit at the kink, within that element's rounding
distance."""
import numpy as np

from oracle import losses_ref

# A shared kink sign that the oracle's own normals would take the other way must sit at the kink:
# |v| (a component of normal - centroid, or a dot of two unit centroids: quantities of scale 1) no
# larger than the distance the two sides' normals put between them, and below this absolute scale
# (2.5x the largest normal angle measured in round 5, 4e-3 rad in bf16).
KINK_ABS = 1e-2


def kink_flips(nh_valid, no_valid, labels):
    """Every kink branch on which the two sides' normals (the same labels) disagree: the oracle's own
    |v|, the HIP side's |v| and that element's rounding distance — |v_o - v_h| <= |dn| + |dc| for an
    L1 component (the normal's chord plus its centroid's), |dc_i| + |dc_j| for a centroid dot product.
    Returns a list of dicts (kind, |v_o|, |v_h|, bound)."""
    vo_ort, vo_l1, co = losses_ref.kink_values(no_valid, labels)
    vh_ort, vh_l1, ch = losses_ref.kink_values(nh_valid, labels)
    dc = np.linalg.norm(co - ch, axis=1)
    out = []
    for i, (a, b) in enumerate(((0, 1), (0, 2), (1, 2))):
        if np.sign(vo_ort[i]) != np.sign(vh_ort[i]):
            out.append({"kind": f"ort{a}{b}", "v_o": abs(vo_ort[i]), "v_h": abs(vh_ort[i]), "bound": dc[a] + dc[b]})
    lab = np.abs(np.asarray(labels))
    for k in range(3):
        sel = lab == k + 1
        dn = np.linalg.norm(np.asarray(nh_valid, np.float64)[sel] - np.asarray(no_valid, np.float64)[sel], axis=1)
        rows, cols = np.nonzero(np.sign(vo_l1[k]) != np.sign(vh_l1[k]))
        for r, c in zip(rows, cols):
            out.append({"kind": f"l1c{k + 1}", "v_o": abs(vo_l1[k][r, c]), "v_h": abs(vh_l1[k][r, c]),
                        "bound": dn[r] + dc[k]})
    return out


def check_kink_flips(flips):
    for f in flips:
        lim = min(1.01 * f["bound"] + 1e-12, KINK_ABS)
        assert f["v_o"] <= lim and f["v_h"] <= lim, ("shared kink sign away from the kink", f, lim)
