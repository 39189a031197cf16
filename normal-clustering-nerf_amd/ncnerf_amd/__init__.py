"""ncnerf_amd — MI355X (gfx950) hot path of the normal-clustering NeRF (nikola3794/normal-clustering-nerf).

Drop-in surface (mirrors the reference module names):
  ncnerf_amd.vren              <- models/csrc (the `vren` extension)
  ncnerf_amd.custom_functions  <- models/custom_functions.py
  ncnerf_amd.rendering.render  <- models/rendering.py
  ncnerf_amd.ngp_mt.NGPMT      <- models/ngp_mt.py (+ tiny-cuda-nn)
  ncnerf_amd.losses.NeRFMTLoss <- losses.py (+ faiss)
All compute goes through libncnerf.so (C ABI: include/ncnerf.h); there is no CPU fallback.
"""
from . import _lib  # noqa: F401

__all__ = ["vren", "custom_functions", "rendering", "ngp_mt", "losses", "optim", "trainer", "synthetic",
           "distributed"]
