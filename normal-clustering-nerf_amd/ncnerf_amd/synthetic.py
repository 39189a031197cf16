"""Synthetic Hypersim-shaped training inputs; no dataset is available offline.

* scene: ai_001_001 box normalised to [-0.476,0.476] x [-0.415,0.415] x [-0.293,0.293]
  (scene_boundaries.json via hypersim.py:63-69), camera centres uniform in the normalised camera box,
  yaw U[0,2pi), pitch U[-20deg,10deg], 1024x768 pinhole, hfov 60deg, unit-norm directions
  (cam_model.py:192-194), rays_o = camera centre, rays_d = R @ dir_cam (ray_utils.py:45-71);
* batches: `all_images_triang_patch` — R/64 random 8x8 patches, each from a random camera
  (datasets/base.py:142-171), so the patch triangle indices of losses.py:307-313 apply;
* occupancy: C=1, G=128 bitfield of a procedural Manhattan room — 8-voxel walls/floor/ceiling on
  the scene box plus 32 random axis-aligned boxes of 4-16 voxels (seed 0).  The wall thickness
  stands in for the thick occupied shell a partly trained density grid has around surfaces; it
  gives ~72 marched samples per ray, inside the 64-200 band SURVEY §8(d) targets.
This is input generation (the reference's dataset role), not part of the measured hot path.
"""
import math

import numpy as np
import torch

SCENE_MIN = np.array([-0.476, -0.415, -0.293], np.float32)
SCENE_MAX = np.array([0.476, 0.415, 0.293], np.float32)
CAM_MIN = np.array([-0.404, -0.367, 0.010], np.float32)
CAM_MAX = np.array([0.453, 0.392, 0.119], np.float32)
IMG_W, IMG_H, HFOV = 1024, 768, 1.0472
PATCH = 8


def _expand_bits(v):
    v = v.astype(np.uint64)
    v = (v * 0x00010001) & 0xFF0000FF
    v = (v * 0x00000101) & 0x0F00F00F
    v = (v * 0x00000011) & 0xC30C30C3
    v = (v * 0x00000005) & 0x49249249
    return v.astype(np.uint32)


def morton3d_np(x, y, z):
    return _expand_bits(x) | (_expand_bits(y) << 1) | (_expand_bits(z) << 2)


def room_occupancy(G=128, n_boxes=32, seed=0, scale=0.5, wall=8):
    """Boolean (G,G,G) occupancy [x][y][z] of the procedural room."""
    rng = np.random.default_rng(seed)
    occ = np.zeros((G, G, G), bool)
    to_vox = lambda v: np.clip(np.floor((v + scale) / (2 * scale) * G).astype(int), 0, G - 1)
    lo, hi = to_vox(SCENE_MIN), to_vox(SCENE_MAX)
    t = wall
    occ[lo[0]:hi[0] + 1, lo[1]:hi[1] + 1, lo[2]:lo[2] + t] = True  # floor
    occ[lo[0]:hi[0] + 1, lo[1]:hi[1] + 1, hi[2] - t + 1:hi[2] + 1] = True  # ceiling
    occ[lo[0]:lo[0] + t, lo[1]:hi[1] + 1, lo[2]:hi[2] + 1] = True
    occ[hi[0] - t + 1:hi[0] + 1, lo[1]:hi[1] + 1, lo[2]:hi[2] + 1] = True
    occ[lo[0]:hi[0] + 1, lo[1]:lo[1] + t, lo[2]:hi[2] + 1] = True
    occ[lo[0]:hi[0] + 1, hi[1] - t + 1:hi[1] + 1, lo[2]:hi[2] + 1] = True
    for _ in range(n_boxes):
        size = rng.integers(4, 17, 3)
        start = [rng.integers(lo[k] + t, max(lo[k] + t + 1, hi[k] - t - size[k])) for k in range(3)]
        occ[start[0]:start[0] + size[0], start[1]:start[1] + size[1], start[2]:start[2] + size[2]] = True
    return occ


def occupancy_to_grid(occ):
    """(G,G,G) bool -> density grid (1, G^3) float32 indexed by morton3D(x,y,z) (ngp_mt.py layout)."""
    G = occ.shape[0]
    grid = np.zeros((1, G ** 3), np.float32)
    x, y, z = np.nonzero(occ)
    grid[0, morton3d_np(x, y, z)] = 1.0
    return grid


def bitfield_np(occ):
    grid = occupancy_to_grid(occ)[0]
    bits = (grid > 0.5).reshape(-1, 8)
    return np.packbits(bits, axis=1, bitorder="little").reshape(-1)


def make_cameras(n_cams=100, seed=0):
    """c2w (n,3,4): columns right, down, forward (OpenCV camera), z-up world."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(CAM_MIN, CAM_MAX, size=(n_cams, 3)).astype(np.float32)
    yaw = rng.uniform(0, 2 * math.pi, n_cams)
    pitch = rng.uniform(math.radians(-20), math.radians(10), n_cams)
    f = np.stack([np.cos(pitch) * np.cos(yaw), np.cos(pitch) * np.sin(yaw), np.sin(pitch)], -1)
    up = np.array([0, 0, 1.0])
    right = np.cross(f, up)
    right /= np.linalg.norm(right, axis=1, keepdims=True)
    down = np.cross(f, right)
    R = np.stack([right, down, f], -1)  # columns
    return np.concatenate([R, c[:, :, None]], -1).astype(np.float32)


def camera_directions():
    """Unit-norm pixel directions (H*W, 3) in camera coordinates (pinhole, pixel centres)."""
    fx = (IMG_W / 2) / math.tan(HFOV / 2)
    u, v = np.meshgrid(np.arange(IMG_W, dtype=np.float32) + 0.5, np.arange(IMG_H, dtype=np.float32) + 0.5)
    d = np.stack([(u - IMG_W / 2) / fx, (v - IMG_H / 2) / fx, np.ones_like(u)], -1).reshape(-1, 3)
    return (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)


def _gt_color(rays_d):
    """View-only target (gt="direction"): a smooth function of the ray direction."""
    return (0.5 + 0.4 * np.sin(3.0 * rays_d + np.array([0.0, 2.1, 4.2], np.float32))).astype(np.float32)


_TEX = np.array([[11.0, 7.0, -5.0], [-6.0, 13.0, 8.0], [9.0, -4.0, 12.0]], np.float32)  # texture frequencies
_TEX_PHASE = np.array([0.3, 2.2, 4.1], np.float32)


def texture_rgb(p, lo=0.1, hi=0.9, freq=1.0):
    """Albedo of the room surfaces at points p (N,3): smooth procedural texture in [lo, hi]; freq
    scales the texture frequencies (0: a constant albedo per channel)."""
    return (0.5 * (hi + lo) + 0.5 * (hi - lo) * np.sin(p @ (freq * _TEX).T + _TEX_PHASE)).astype(np.float32)


def first_hit(occ, rays_o, rays_d, scale=0.5, step_vox=0.25, t_max=2.0, chunk=64):
    """Distance to the first occupied voxel of `occ` along each ray (inf if none inside the
    [-scale, scale]^3 box), by stepping a quarter voxel at a time from t = 0."""
    G = occ.shape[0]
    h = step_vox * 2 * scale / G
    n = rays_o.shape[0]
    t_hit = np.full(n, np.inf, np.float32)
    alive = np.arange(n)
    t0 = 0.0
    while alive.size and t0 < t_max:
        t = t0 + h * np.arange(chunk, dtype=np.float32)
        p = rays_o[alive, None, :] + rays_d[alive, None, :] * t[None, :, None]  # (A, chunk, 3)
        inside = np.all(np.abs(p) < scale, axis=-1)
        v = np.clip(np.floor((p + scale) / (2 * scale) * G).astype(np.int64), 0, G - 1)
        hit = inside & occ[v[..., 0], v[..., 1], v[..., 2]]
        left = ~inside & (t[None, :] > 0)  # outside the box after starting: the ray has left
        first = np.where(hit.any(1), hit.argmax(1), chunk)
        gone = np.where(left.any(1), left.argmax(1), chunk)
        found = first < gone
        t_hit[alive[found]] = t[first[found]]
        alive = alive[~found & (gone == chunk)]
        t0 += h * chunk
    return t_hit


def surface_rgb(occ, rays_o, rays_d, scale=0.5, lo=0.1, hi=0.9, freq=1.0):
    """Target colour of a ray (gt="surface", default): texture_rgb at its first occupied voxel,
    white (the reference's background, rendering.py:232-240) if it hits nothing."""
    t = first_hit(occ, rays_o, rays_d, scale)
    rgb = np.ones((rays_o.shape[0], 3), np.float32)
    m = np.isfinite(t)
    rgb[m] = texture_rgb(rays_o[m] + rays_d[m] * t[m, None], lo, hi, freq)
    return rgb


class SyntheticScene:
    """Holds cameras, directions and the occupancy bitfield; draws patch batches."""

    def __init__(self, G=128, n_cams=100, seed=0, scale=0.5):
        self.G, self.scale = G, scale
        self.occ = room_occupancy(G, seed=seed, scale=scale)
        self.density_grid = occupancy_to_grid(self.occ)
        self.bitfield = bitfield_np(self.occ)
        self.poses = make_cameras(n_cams, seed)
        self.dirs = camera_directions()
        o1 = np.arange(PATCH * PATCH).reshape(PATCH, PATCH)
        self.x1_off, self.x2_off, self.x3_off = o1[1:, 1:].reshape(-1), o1[:-1, 1:].reshape(-1), o1[1:, :-1].reshape(-1)

    def batch(self, n_rays, seed, gt="surface"):
        """A dict like BaseDataset.__getitem__ + get_rays: rays_o, rays_d (R,3) f32, rgb (R,3), patch info.
        gt: "surface" (textured room, the PSNR-parity target), "surface_bright" (the same texture in
        [0.45, 0.95]), "surface_smooth" (that with a quarter of the texture frequency), "surface_flat"
        (a constant albedo per channel) or "direction" (view-only colour)."""
        assert n_rays % (PATCH * PATCH) == 0
        rng = np.random.default_rng(seed)
        n_p = n_rays // (PATCH * PATCH)
        cams = rng.integers(0, len(self.poses), n_p)
        u0 = rng.integers(0, IMG_W - PATCH + 1, n_p)
        v0 = rng.integers(0, IMG_H - PATCH + 1, n_p)
        iy, ix = np.meshgrid(np.arange(PATCH), np.arange(PATCH), indexing="ij")
        pix = ((v0[:, None] + iy.reshape(-1)[None]) * IMG_W + (u0[:, None] + ix.reshape(-1)[None])).reshape(-1)
        cam = np.repeat(cams, PATCH * PATCH)
        dcam = self.dirs[pix]
        P = self.poses[cam]
        rays_d = np.einsum("nij,nj->ni", P[:, :, :3], dcam).astype(np.float32)
        rays_o = P[:, :, 3].astype(np.float32)
        if gt == "surface":
            rgb = surface_rgb(self.occ, rays_o, rays_d, self.scale)
        elif gt == "surface_bright":
            rgb = surface_rgb(self.occ, rays_o, rays_d, self.scale, 0.45, 0.95)
        elif gt == "surface_smooth":
            rgb = surface_rgb(self.occ, rays_o, rays_d, self.scale, 0.45, 0.95, 0.25)
        elif gt == "surface_flat":
            rgb = surface_rgb(self.occ, rays_o, rays_d, self.scale, 0.45, 0.95, 0.0)
        else:
            rgb = _gt_color(rays_d)
        return {"rays_o": rays_o, "rays_d": rays_d, "rgb": rgb, "patch_area": PATCH * PATCH,
                "x1_offsets_local": self.x1_off, "x2_offsets_local": self.x2_off, "x3_offsets_local": self.x3_off}

    def image_rays(self, cam, device=None):
        """Every pixel of camera `cam`'s 1024x768 image (get_rays, ray_utils.py:45-71): the rays of
        the reference's test-time render of one image (validation_step, train_nerf.py:381)."""
        P = self.poses[cam]
        rays_d = (self.dirs @ P[:, :3].T).astype(np.float32)
        rays_o = np.broadcast_to(P[:, 3].astype(np.float32), rays_d.shape).copy()
        if device is None:
            return rays_o, rays_d
        return (torch.from_numpy(rays_o).to(device), torch.from_numpy(np.ascontiguousarray(rays_d)).to(device))

    def torch_batch(self, n_rays, seed, device, gt="surface"):
        """batch() with the per-ray arrays on `device`; the patch offsets stay host arrays (constant
        metadata of the sampling strategy, as the reference's base.py:53-58 keeps them)."""
        b = self.batch(n_rays, seed, gt)
        out = {}
        for k, v in b.items():
            if isinstance(v, np.ndarray) and not k.endswith("_offsets_local"):
                out[k] = torch.from_numpy(np.ascontiguousarray(v)).to(device)
            else:
                out[k] = v
        return out
