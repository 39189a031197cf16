"""Parity of the normal-clustering loss path (ncn_normals_fwd/bwd, ncn_cluster_loss) with the oracle
(oracle/losses_ref.py; the selection/loss restatement is pinned to the reference by tests/golden).

Tolerances: normals |Δ| <= 1e-5; d depth rel-L2 <= 1e-4; k-means centroids |Δ| <= 1e-5 and identical
labels on well-separated (Manhattan) data; losses |Δ| <= 1e-5; d normals rel-L2 <= 1e-3."""
import numpy as np
import pytest
import torch

from oracle import losses_ref
from ncnerf_amd import losses as L

pytestmark = pytest.mark.gpu


def _manhattan_normals(n, seed, noise=0.05, invalid=0):
    rng = np.random.default_rng(seed)
    axes = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], np.float32)
    p = np.array([0.3, 0.05, 0.25, 0.1, 0.25, 0.05])
    x = axes[rng.choice(6, n, p=p)] + rng.normal(0, noise, (n, 3)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    x = x.astype(np.float32)
    if invalid:
        x[rng.choice(n, invalid, replace=False)] = 0.0
        x[0] = np.nan
    return x


def test_normals_fwd_bwd(dev):
    rng = np.random.default_rng(0)
    R = 8192
    x1, x2, x3 = losses_ref.patch_triangle_index(R)
    d = rng.normal(size=(R, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    depth = rng.uniform(0.5, 2.0, R).astype(np.float32)
    o = d.copy()  # quirk q1: rays_o := rays_d
    dt = torch.from_numpy(depth).to(dev).requires_grad_(True)
    idx = {k: torch.from_numpy(v).to(dev) for k, v in zip(("x1", "x2", "x3"), (x1, x2, x3))}
    n = L.extract_normals_from_ray_batch(torch.from_numpy(o).to(dev), torch.from_numpy(d).to(dev), dt, idx)
    gn = torch.from_numpy(rng.normal(size=(len(x1), 3)).astype(np.float32)).to(dev)
    (n * gn).sum().backward()
    dr = torch.from_numpy(depth).requires_grad_(True)
    nr = losses_ref.normals_from_depth(torch.from_numpy(o), torch.from_numpy(d), dr, x1, x2, x3)
    (nr * gn.cpu()).sum().backward()
    np.testing.assert_allclose(n.detach().cpu().numpy(), nr.detach().numpy(), atol=1e-5)
    rel = (dt.grad.cpu() - dr.grad).norm() / dr.grad.norm()
    assert rel < 1e-4, rel


def _degenerate_normals(n, seed):
    """Three exact directions (+ 50 noisy points): the 20 init picks repeat points, so Lloyd rounds
    see empty clusters and take faiss's split path (oracle: 11 distinct final centroids)."""
    rng = np.random.default_rng(seed)
    axes = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1]], np.float32)
    x = axes[rng.choice(3, n)].astype(np.float32)
    x[:50] += rng.normal(0, 0.05, (50, 3)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    return x.astype(np.float32)


@pytest.mark.parametrize("n,invalid", [(6272, 0), (6272, 37), (2000, 5), (6272, -1)])
def test_cluster_loss_parity(dev, n, invalid):
    """invalid = -1: the degenerate set (empty clusters -> split_clusters in the Lloyd rounds)."""
    X = _degenerate_normals(n, seed=5) if invalid < 0 else _manhattan_normals(n, seed=n + invalid, invalid=invalid)
    valid = losses_ref.valid_normals_mask(torch.from_numpy(X)).numpy()
    Xv = X[valid]
    C, a = losses_ref.spherical_kmeans(Xv, K=20, niter=20, seed=1234)
    lab, cn = losses_ref.cluster_select(C, a, 0.99)
    xt = torch.from_numpy(Xv).requires_grad_(True)
    ort, cdot, cl1 = losses_ref.cluster_losses(xt, torch.from_numpy(lab))
    w = (2e-3, 3e-3, 5e-3)
    (w[0] * ort + w[1] * cdot + w[2] * cl1).backward()
    Xd = torch.from_numpy(X).to(dev).requires_grad_(True)
    terms, labels, cents, raw = L.cluster_losses(Xd, K=20, niter=20, seed=1234, t_similar=0.99, w=w)
    terms.sum().backward()
    np.testing.assert_allclose(cents.cpu().numpy(), C, atol=1e-5)
    lab_d = labels.cpu().numpy()
    assert np.array_equal(lab_d[valid], lab)
    assert np.all(lab_d[~valid] == -9)
    np.testing.assert_allclose(terms.detach().cpu().numpy(), [w[0] * ort.item(), w[1] * cdot.item(), w[2] * cl1.item()],
                               rtol=1e-4, atol=1e-8)
    g_ref = torch.zeros(n, 3)
    g_ref[torch.from_numpy(valid)] = xt.grad
    rel = (Xd.grad.cpu() - g_ref).norm() / g_ref.norm()
    assert rel < 1e-3, rel


def test_cluster_loss_too_few(dev):
    X = _manhattan_normals(12, seed=0)
    Xd = torch.from_numpy(X).to(dev)
    terms, labels, cents, raw = L.cluster_losses(Xd, K=20)
    assert float(terms.abs().sum()) == 0.0 and float(raw[3]) == 12


def _depth_batch(dev, R, seed):
    """Depths of a tilted plane seen through patch rays, so the normals form a few clusters."""
    rng = np.random.default_rng(seed)
    x1, x2, x3 = losses_ref.patch_triangle_index(R)
    d = rng.normal(size=(R, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    depth = rng.uniform(0.5, 2.0, R).astype(np.float32)
    idx = {k: torch.from_numpy(v).to(dev) for k, v in zip(("x1", "x2", "x3"), (x1, x2, x3))}
    return torch.from_numpy(d).to(dev), torch.from_numpy(depth).to(dev), idx


def test_fused_normals_cluster_matches_unfused(dev):
    """normals_cluster_losses (one autograd node, device-side term weights in ncn_normals_bwd) must
    give the same terms and depth gradient as extract_normals_from_ray_batch + cluster_losses.
    Tolerance: terms |d| <= 1e-7 (same kernels), d depth rel-L2 <= 1e-5 (summation order)."""
    d, depth, idx = _depth_batch(dev, 8192, 3)
    w = (2e-3, 3e-3, 5e-3)
    g = torch.tensor([1.0, 0.5, 2.0], device=dev)
    d1 = depth.clone().requires_grad_(True)
    n = L.extract_normals_from_ray_batch(d, d, d1, idx)
    t1, lab1, c1, _ = L.cluster_losses(n, w=w)
    (t1 * g).sum().backward()
    d2 = depth.clone().requires_grad_(True)
    t2, n2, lab2, c2, _ = L.normals_cluster_losses(d, d, d2, idx, w=w)
    (t2 * g).sum().backward()
    torch.testing.assert_close(n2, n.detach(), rtol=0, atol=0)
    assert torch.equal(lab1, lab2)
    torch.testing.assert_close(t2, t1.detach(), rtol=0, atol=1e-7)
    rel = (d2.grad - d1.grad).norm() / d1.grad.norm().clamp_min(1e-30)
    assert rel < 1e-5, rel


@pytest.mark.parametrize("R,bad", [(8192, False), (1000, False), (4096, True)])
def test_photo_losses(dev, R, bad):
    """ncn_photo_loss_fwd/bwd vs the torch expressions of losses.py:349-362 (+ validity filter).
    Tolerance: values rel 1e-5, gradients rel 1e-5; a NaN rgb zeroes that term and its gradient."""
    gen = torch.Generator(device="cpu").manual_seed(R)
    rgb = torch.rand(R, 3, generator=gen).to(dev)
    gt = torch.rand(R, 3, generator=gen).to(dev)
    op = torch.rand(R, generator=gen).to(dev)
    if bad:
        rgb[7, 1] = float("nan")
    a, b = rgb.clone().requires_grad_(True), op.clone().requires_grad_(True)
    l_rgb, l_op = L.photo_losses(a, gt, b, 1e-3)
    (2.0 * l_rgb + 3.0 * l_op).backward()
    a2, b2 = rgb.clone().requires_grad_(True), op.clone().requires_grad_(True)
    r2 = ((a2 - gt) ** 2).mean()
    o = b2 + 1e-10
    e2 = 1e-3 * (-o * torch.log(o)).mean()
    ok = bool(torch.isfinite(r2))
    (2.0 * (r2 if ok else 0 * r2.nan_to_num()) + 3.0 * e2).backward()
    if ok:
        torch.testing.assert_close(l_rgb, r2.detach(), rtol=1e-5, atol=0)
        torch.testing.assert_close(a.grad, a2.grad, rtol=1e-5, atol=1e-12)
    else:
        assert float(l_rgb) == 0.0 and float(a.grad.abs().sum()) == 0.0
    torch.testing.assert_close(l_op, e2.detach(), rtol=1e-5, atol=0)
    torch.testing.assert_close(b.grad, b2.grad, rtol=1e-5, atol=1e-12)


def test_fused_nerf_loss_matches_unfused(dev):
    """NeRFMTLoss in the reference configuration through the one-node path (_NeRFLossFused: photo +
    normals + clustering forward, ONE backward kernel gathering dL/ddepth per ray) against the
    multi-node path (taken when the patch offsets are device tensors).  Both with the device step
    (graph path) and a host step.  Tolerance: losses rel 1e-6, gradients rel-L2 1e-5 (the
    depth gradient is gathered per ray instead of accumulated with atomics)."""
    from ncnerf_amd.synthetic import SyntheticScene
    from ncnerf_amd.trainer import HYPERSIM_HPARAMS
    R = 8192
    d, depth, _ = _depth_batch(dev, R, 5)
    rng = np.random.default_rng(6)
    rgb = torch.from_numpy(rng.random((R, 3), dtype=np.float32)).to(dev)
    op = torch.from_numpy(rng.random(R, dtype=np.float32)).to(dev)
    gt = torch.from_numpy(rng.random((R, 3), dtype=np.float32)).to(dev)
    sc = SyntheticScene()
    host_off = dict(x1_offsets_local=sc.x1_off, x2_offsets_local=sc.x2_off, x3_offsets_local=sc.x3_off)
    dev_off = {k: torch.from_numpy(v).to(dev) for k, v in host_off.items()}
    for step in (1800, torch.tensor(1800, device=dev)):
        out = []
        for off in (dev_off, host_off):
            loss = L.NeRFMTLoss(HYPERSIM_HPARAMS)
            a, b, c = (t.clone().requires_grad_(True) for t in (rgb, op, depth))
            pred = dict(rgb=a, opacity=b, depth=c, rays_o=d, rays_d=d)
            ld = loss(pred, dict(rgb=gt, patch_area=64, **off), global_step=step)
            ld["total"].backward()
            out.append(({k: float(v) for k, v in ld.items()}, a.grad, b.grad, c.grad))
        (l0, *g0), (l1, *g1) = out
        assert set(l0) == set(l1)
        for k in l0:
            np.testing.assert_allclose(l1[k], l0[k], rtol=1e-6, atol=1e-9, err_msg=k)
        assert l1["norm_D_C_ort_dot"] > 0
        for x, y in zip(g0, g1):
            rel = float((y - x).norm() / x.norm().clamp_min(1e-30))
            assert rel < 1e-5, rel


def test_cluster_after_unclustered_call(dev):
    """A launch with too few normals must not leave the next clustered launch reading an older
    launch's Lloyd partials (the tag sequence advances on every launch)."""
    for seed in (3, 4):
        X = _manhattan_normals(6272, seed=seed)
        L.cluster_losses(torch.from_numpy(X).to(dev), K=20, niter=20, seed=1234)
        L.cluster_losses(torch.from_numpy(_manhattan_normals(12, seed=seed)).to(dev), K=20)
    X = _manhattan_normals(6272, seed=6272)  # the data of test_cluster_loss_parity[6272-0]
    valid = losses_ref.valid_normals_mask(torch.from_numpy(X)).numpy()
    C, a = losses_ref.spherical_kmeans(X[valid], K=20, niter=20, seed=1234)
    _, labels, cents, _ = L.cluster_losses(torch.from_numpy(X).to(dev), K=20, niter=20, seed=1234, t_similar=0.99)
    np.testing.assert_allclose(cents.cpu().numpy(), C, atol=1e-5)


_STATUS_CHILD = r"""
import os, sys
sys.path[:0] = [os.path.join(sys.argv[1], "normal-clustering-nerf_amd"), sys.argv[1]]
import numpy as np, torch
from ncnerf_amd import losses as L, _lib
rng = np.random.default_rng(0)
x = rng.normal(size=(6272, 3)).astype(np.float32)
x /= np.linalg.norm(x, axis=1, keepdims=True)
L.cluster_losses(torch.from_numpy(x).cuda(), K=20, niter=20)
torch.cuda.synchronize()
try:
    L.check_cluster_status()
except _lib.NcnError as e:
    print("RAISED", e)
    sys.exit(0)
print("NOT RAISED")
sys.exit(1)
"""


def test_cluster_status_word(dev):
    """The clustering kernel's sticky error word reaches the caller: clean after normal launches;
    a diagnostic build whose barrier / hand-off spin limits are 1 (libncnerf_diag_kmspin.so) sets it
    in a real launch and check_cluster_status raises; a set word raises on the product library."""
    import os
    import subprocess
    import sys
    from ncnerf_amd import _lib
    L.check_cluster_status()  # the launches of the tests above left it clear
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    diag = os.path.join(root, "normal-clustering-nerf_amd", "ncnerf_amd", "libncnerf_diag_kmspin.so")
    assert os.path.exists(diag), "build the diagnostic library (make -C normal-clustering-nerf_amd)"
    r = subprocess.run([sys.executable, "-c", _STATUS_CHILD, root], env=dict(os.environ, NCN_LIB_PATH=diag),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "RAISED" in r.stdout, r.stdout + r.stderr[-2000:]
    # product library: a set word is reported
    x = torch.from_numpy(_manhattan_normals(512, 3)).to(dev)
    L.cluster_losses(x, K=20, niter=20)
    ws = L._WS[(str(dev), 20)]
    off = int(_lib.lib().ncn_cluster_status_offset(20))
    ws.view(torch.int32)[off] = 1
    with pytest.raises(_lib.NcnError):
        L.check_cluster_status(dev)
    ws.view(torch.int32)[off] = 0
    L.check_cluster_status(dev)


_DROP_CHILD = r"""
import os, sys
sys.path[:0] = [os.path.join(sys.argv[1], "normal-clustering-nerf_amd"), sys.argv[1]]
import torch
from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers
from ncnerf_amd.synthetic import SyntheticScene
from ncnerf_amd.rendering import render
from ncnerf_amd.trainer import Trainer
from ncnerf_amd import losses as L, _lib
dev = torch.device("cuda", 0)
scene = SyntheticScene()
torch.manual_seed(0)
model = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
model.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
with torch.no_grad():  # a non-trivial field so that the depth (and the normals) carry gradient
    model.flat_params()[: model._n_table].uniform_(-0.5, 0.5, generator=torch.Generator(device=dev).manual_seed(5))
batch = scene.torch_batch(2048, seed=11, device=dev)
noise = torch.rand(2048, generator=torch.Generator().manual_seed(12)).to(dev)
tr = Trainer(model, use_graph=False)
out = {}
for step in [int(s) for s in sys.argv[3].split(",")]:
    model.flat_grad().zero_()
    kw = dict(tr.render_kwargs, global_step=step, march_noise=noise)
    res = render(model, batch["rays_o"], batch["rays_d"], **kw)
    loss_d = tr.loss(res, batch, global_step=step)
    loss_d["total"].backward()
    torch.cuda.synchronize()
    out[step] = {"grad": model.flat_grad().cpu().clone(),
                 "losses": {k: float(v) for k, v in loss_d.items() if torch.is_tensor(v) and v.numel() == 1}}
try:
    L.check_cluster_status()
    out["status"] = 0
except _lib.NcnError:
    out["status"] = 1
torch.save(out, sys.argv[2])
"""


def test_cluster_timeout_drops_cluster_terms(dev, tmp_path):
    """A clustering launch whose grid barrier / hand-off timed out must not train on its partial
    sums: the kernel drops the cluster terms (losses 0, no normal gradient) as the reference's
    validity filter drops an invalid term (losses.py:246-262).  The diagnostic library (spin limits
    1: every barrier times out) at a step past the weight ramp (3000) must give the gradient of the
    photometric terms alone — the product library's gradient at step 400, where the ramp holds the
    cluster weights at 0 (losses.py:217) — while the product library's own gradient at step 3000
    differs from that (the cluster terms do contribute there)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    diag = os.path.join(root, "normal-clustering-nerf_amd", "ncnerf_amd", "libncnerf_diag_kmspin.so")
    assert os.path.exists(diag), "build the diagnostic library (make -C normal-clustering-nerf_amd)"
    runs = {}
    for name, lib, steps in (("prod", None, "400,3000"), ("diag", diag, "3000")):
        o = str(tmp_path / f"{name}.pt")
        env = dict(os.environ)
        if lib:
            env["NCN_LIB_PATH"] = lib
        r = subprocess.run([sys.executable, "-c", _DROP_CHILD, root, o, steps], env=env, capture_output=True,
                           text=True, timeout=180)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
        runs[name] = torch.load(o, weights_only=True)
    prod, diag_r = runs["prod"], runs["diag"]
    assert prod["status"] == 0 and diag_r["status"] == 1
    photo, full, dropped = prod[400]["grad"], prod[3000]["grad"], diag_r[3000]["grad"]
    lo = diag_r[3000]["losses"]
    for k in ("norm_D_C_ort_dot", "norm_D_C_centr_dot", "norm_D_C_centr_L1"):
        assert lo[k] == 0.0, (k, lo[k])
    assert lo["total"] == float(np.float32(lo["rgb"]) + np.float32(lo["opacity"]))  # (the kernel's f32 sum)
    assert prod[3000]["losses"]["norm_D_C_centr_L1"] > 0
    assert torch.isfinite(dropped).all()
    rel = lambda a, b: float((a - b).norm() / b.norm())
    print(f"timed-out step vs photometric-only gradient: rel-L2 {rel(dropped, photo):.2e}; "
          f"full step vs photometric-only: {rel(full, photo):.2e}")
    assert rel(dropped, photo) < 1e-5
    assert rel(full, photo) > 1e-3


def test_cluster_coresidency_refuses(dev):
    """The clustering kernel's 16 workgroups meet at grid barriers, so all of them must be resident
    at once.  ncn_cluster_coresidency reports how many fit beside `busy` CUs of
    concurrent work; the split step checks it for its rgb pass (one workgroup per CU) before it is
    captured, and refuses — raises, launching nothing — when the clustering could not stay resident,
    instead of spinning into the barrier timeout."""
    import ctypes
    from ncnerf_amd import _lib
    from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers
    from ncnerf_amd.split_step import SPLIT_BLOCKS, SplitStep
    from ncnerf_amd.trainer import Trainer
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    cap = ctypes.c_int(0)
    assert _lib.lib().ncn_cluster_coresidency(20, 0, ctypes.byref(cap)) == 0
    per_cu = cap.value // cus
    assert per_cu >= 1 and cap.value >= 16, (cap.value, cus)
    assert _lib.lib().ncn_cluster_coresidency(20, SPLIT_BLOCKS, ctypes.byref(cap)) == 0
    assert cap.value == (cus - SPLIT_BLOCKS) * per_cu >= 16
    busy = cus - (16 - 1) // per_cu  # leaves fewer free CUs than 16 workgroups need
    rc = _lib.lib().ncn_cluster_coresidency(20, busy, ctypes.byref(cap))
    assert rc != 0 and cap.value < 16, (rc, cap.value)
    assert "cannot all be resident" in _lib.lib().ncn_last_error().decode()
    m = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
    tr = Trainer(m, update_grid=False, use_graph=True)
    assert SplitStep(tr).cluster_capacity >= 16
    with pytest.raises(_lib.NcnError, match="cannot all be resident"):
        SplitStep(tr, rgb_blocks=busy)
