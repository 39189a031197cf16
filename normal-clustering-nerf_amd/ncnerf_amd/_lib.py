"""ctypes binding of libncnerf.so (the C ABI declared in include/ncnerf.h).

This is the only place Python talks to the HIP kernels.  There is NO CPU fallback: if the library
is missing, or a kernel is called with a CPU tensor, the call raises.  Tensors are passed as raw
device pointers and sizes, on torch's *current* HIP stream (never the legacy default stream).
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NCN_LIB_PATH") or os.path.join(_HERE, "libncnerf.so")  # (override: diagnostics)

P = ctypes.c_void_p
I64 = ctypes.c_int64
I32 = ctypes.c_int
U32 = ctypes.c_uint32
F32 = ctypes.c_float
F64 = ctypes.c_double
AMP_INIT_SCALE = 65536.0  # NCN_AMP_INIT_SCALE (include/ncnerf.h): torch GradScaler's init_scale
U64 = ctypes.c_uint64

# name -> argtypes (stream last); every function returns int (hipError_t)
SIGNATURES = {
    "ncn_grad_pack_f16": [P, I64, P, I32, P, P],
    "ncn_grad_unpack_f16": [P, I64, P, P, P],
    "ncn_morton3D": [P, I64, P, P],
    "ncn_morton3D_invert": [P, I64, P, P],
    "ncn_packbits": [P, I64, F32, P, P],
    "ncn_ray_aabb_intersect": [P, P, I64, P, P, I64, I32, P, P, P, P],
    "ncn_ray_aabb_intersect_near": [P, P, I64, P, P, I64, I32, F32, P, P, P, P],
    "ncn_march_train_walk": [P, P, P, P, I64, P, I32, F32, F32, I32, I32, P, P, P, P, P],
    "ncn_march_train_scan": [P, I64, P, P, P],
    "ncn_march_train_fused_work_bytes": [I64],
    "ncn_march_train_fused": [P, P, I64, F32, F32, F32, F32, F32, F32, F32, P, U64, P, P, I32, F32, I32, I32, P, P, P,
                              P, P, P, P, P, P, P, P],
    "ncn_march_train_pack": [P, P, I64, I32, P, P, P, P, P, P, P, P],
    "ncn_segment_csr": [P, P, P, P, I64, P, P, P],
    "ncn_march_test": [P, P, P, P, I64, P, I32, F32, F32, I32, I32, I32, P, P, P, P, P, P],
    "ncn_composite_train_fw": [P, P, P, P, P, I64, I64, I32, F32, P, P, P, P, P, P],
    "ncn_composite_train_bw": [P, P, P, P, P, P, P, P, P, P, I64, I64, I32, P, P, P, F32, P, P, P],
    "ncn_composite_train_fw_bg": [P, P, P, P, P, I64, I64, I32, F32, P, P, P, P, P, F32, P, P],
    "ncn_count_samples": [P, I64, P, P, P, P],
    "ncn_step_inputs": [I32, P, P, P, P, I64, P, I32, P],
    "ncn_composite_train_bw_bg": [P, P, P, P, P, P, P, P, P, P, I64, I64, I32, P, P, P, F32, F32, P, P, P],
    "ncn_test_compact": [P, P, P, I64, I32, P, P, P, P, P],
    "ncn_composite_test_fw_compact": [P, P, P, P, P, P, I64, I32, I32, F32, P, P, P, P, P],
    "ncn_test_loop_march": [P, P, P, P, I64, P, I32, F32, F32, I32, I32, P, P, P, P, P, P, P],
    "ncn_test_loop_index": [P, I64, P, P, P],
    "ncn_test_loop_composite": [P, P, P, P, P, P, I64, P, I32, F32, P, P, P, P, P],
    "ncn_test_loop_next": [P, P, I64, P, P, I32, I32, I32, P],
    "ncn_composite_test_fw": [P, P, P, P, P, I64, I32, I32, F32, P, P, P, P, P],
    "ncn_field_pack_weights": [P, P, I32, P],
    "ncn_field_pack_map": [P, P],
    "ncn_field_sort_windows": [P, I64, P, F32, F32, P, P],
    "ncn_field_fwd": [P, P, I64, P, P, P, P, F32, F32, P, I32, I32, P, P, P, P],
    "ncn_field_bwd_blocks": [I64],
    "ncn_field_bwd_dE_floats": [I64],
    "ncn_field_bwd": [P, P, I64, P, P, P, F32, F32, P, I32, P, P, P, P, P, P, P, P, P],
    "ncn_field_bwd_mlp": [P, P, I64, P, P, P, I32, P, P, P, P, P, P, P, P],
    "ncn_field_bwd_stash_floats": [I64],
    "ncn_field_bwd_part_blocks": [I64, I32],
    "ncn_field_reduce_wgrad_parts": [P, I32, I32, P, P],
    "ncn_field_bwd_mlp_part": [P, P, I64, P, P, P, I32, P, P, P, P, P, I32, I32, P, P, P, P, P],
    "ncn_field_scatter_positions": [P, I64, P, P, P],
    "ncn_field_scatter": [P, I64, P, P, P, F32, F32, P, P, I32, I32, I32, P, P],
    "ncn_field_scatter_wgrad": [P, I64, P, P, P, F32, F32, P, P, I32, I32, I32, P, P, I32, I32, P, P],
    "ncn_field_reduce_wgrad": [P, I32, P, P],
    "ncn_normals_fwd": [P, P, P, P, P, P, I64, P, P],
    "ncn_normals_bwd": [P, P, P, P, P, P, I64, P, P, P, P],
    "ncn_photo_loss_fwd": [P, P, P, I64, F32, P, P],
    "ncn_photo_normals_fwd": [P, P, P, I64, F32, P, P, P, P, P, P, P, I64, P, P],
    "ncn_photo_normals_count_fwd": [P, P, P, I64, F32, P, P, P, P, P, P, P, I64, P, P, I64, P, P, P, P],
    "ncn_photo_loss_bwd": [P, P, P, I64, F32, P, P, P, P, P],
    "ncn_cluster_workspace_words": [I32],
    "ncn_cluster_status_offset": [I32],
    "ncn_cluster_coresidency": [I32, I32, P],
    "ncn_kmeans_plan_words": [I32, I32],
    "ncn_kmeans_plan_fill": [I32, I32, U32, P],
    "ncn_cluster_loss": [P, I64, I32, I32, P, F32, F32, F32, F32, P, P, F32, F32, P, P, P, P, P, P, P],
    "ncn_nerf_loss_bwd": [P, P, P, I64, F32, P, P, P, P, P, P, P, P, P, P, P],
    "ncn_sumsq": [P, I64, P, P, P],
    "ncn_adam": [P, P, P, P, I64, P, F32, F32, F32, F32, F32, F32, I32, P, P, P],
    "ncn_adam_step": [P, P, P, P, I64, I64, F32, F32, F32, F64, F64, F32, F32, F32, P, P, P, I32, P, P, P],
    "ncn_adam_step_packed": [P, P, P, P, I64, I64, F32, F32, F32, F64, F64, F32, F32, F32, P, P, P, I32, P, P,
                             P, I64, P, I32, P],
    "ncn_adam_step_work_floats": [],
    "ncn_distortion_loss_fw": [P, P, P, P, I64, P, P, P, P],
    "ncn_distortion_loss_bw": [P, P, P, P, P, P, P, I64, P, P],
    "ncn_grid_work_bytes": [],
    "ncn_grid_sample": [P, I64, I32, F32, F32, F32, I64, I32, U64, F32, P, P, P, P, P, P],
    "ncn_grid_apply": [P, P, P, P, I64, F32, P, P],
    "ncn_grid_packbits": [P, I64, F64, P, P, P, P],
}

_lib = None

# Optional per-kernel timing: when TIMING is a dict, `call` brackets each launch of the entry points
# that are keys of TIMING with HIP events on the current stream (the stream the kernel runs on) and
# appends (start, end) to TIMING[name].  A GPU spin (torch.cuda._sleep) is queued in front of the
# start event so the device is still busy while Python issues the launch: the events then bracket
# the kernel itself, not the ~6 us of host-side launch latency (checked against rocprofv3).
TIMING = None
TIMING_SPIN_CYCLES = 60000


class NcnError(RuntimeError):
    pass


def lib():
    """Load libncnerf.so (after torch's HIP runtime, so both share one libamdhip64)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NcnError(f"libncnerf.so not found at {LIB_PATH}: run __graft_entry__.build() "
                           f"(make -C normal-clustering-nerf_amd)")
        L = ctypes.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = ctypes.c_int
        L.ncn_cluster_workspace_words.restype = ctypes.c_int64
        L.ncn_cluster_status_offset.restype = ctypes.c_int64
        L.ncn_kmeans_plan_words.restype = ctypes.c_int64
        L.ncn_field_bwd_dE_floats.restype = ctypes.c_int64
        L.ncn_field_bwd_stash_floats.restype = ctypes.c_int64
        L.ncn_adam_step_work_floats.restype = ctypes.c_int64
        L.ncn_grid_work_bytes.restype = ctypes.c_int64
        L.ncn_march_train_fused_work_bytes.restype = ctypes.c_int64
        L.ncn_last_error.argtypes = []
        L.ncn_last_error.restype = ctypes.c_char_p
        L.ncn_version.restype = ctypes.c_int
        _lib = L
    return _lib


def exported_symbols():
    return list(SIGNATURES) + ["ncn_last_error", "ncn_version"]


def call(name, *args):
    if TIMING is not None and name in TIMING:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(TIMING_SPIN_CYCLES)
        e0.record()
        rc = getattr(lib(), name)(*args)
        e1.record()
        TIMING[name].append((e0, e1))
    else:
        rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().ncn_last_error().decode(errors="replace")
        raise NcnError(f"{name} failed (hipError {rc}): {msg}")
    return rc


def stream():
    return P(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    """Raw device pointer of a CUDA tensor (None -> NULL)."""
    if t is None:
        return P(None)
    return P(t.data_ptr())


def step_inputs(srcs, dsts, step_dev, step, flag_dev=None, flag=0):
    """ncn_step_inputs: copy each srcs[i] into dsts[i] (contiguous CUDA tensors of equal size), write
    `step` into the int64 device scalar step_dev and `flag` into the int32 flag_dev, in one launch."""
    n = len(srcs)
    VP = ctypes.c_void_p * max(n, 1)
    src = VP(*[s.data_ptr() for s in srcs])
    dst = VP(*[d.data_ptr() for d in dsts])
    nb = (ctypes.c_int64 * max(n, 1))(*[s.numel() * s.element_size() for s in srcs])
    return call("ncn_step_inputs", I32(n), ctypes.cast(src, P), ctypes.cast(dst, P), ctypes.cast(nb, P),
                ptr(step_dev), I64(int(step)), ptr(flag_dev), I32(int(flag)), stream())


def check_input(t, name):
    """The reference's CHECK_INPUT (models/csrc/include/utils.h:4-6)."""
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")


def check_dtype(t, dtype, name):
    if t.dtype != dtype:
        raise RuntimeError(f"{name} must be {dtype} (got {t.dtype})")
