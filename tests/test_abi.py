"""The C ABI library: loads on CPU-only hosts and exports every symbol include/ncnerf.h declares
(no compute calls without a GPU)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ncnerf.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ncn_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_hot_path():
    syms = declared_symbols()
    for s in ("ncn_ray_aabb_intersect", "ncn_march_train_walk", "ncn_march_train_scan", "ncn_march_train_pack",
              "ncn_composite_train_fw", "ncn_composite_train_bw", "ncn_field_fwd", "ncn_field_bwd", "ncn_field_sort_windows",
              "ncn_normals_fwd", "ncn_cluster_loss", "ncn_adam", "ncn_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from ncnerf_amd import _lib
    L = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    from ncnerf_amd import _lib
    bound = set(_lib.exported_symbols())
    assert set(declared_symbols()) <= bound, set(declared_symbols()) - bound
    L = _lib.lib()
    assert L.ncn_version() >= 1
    assert L.ncn_last_error() is not None


def test_library_is_gfx950_code_object():
    from ncnerf_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data
