"""ctypes binding of libdpft_ic.so (C ABI: include/dpft_ic.h).

The library is loaded only after torch, so its `libamdhip64.so.7` dependency
resolves to the HIP runtime torch already mapped (one runtime, one set of
streams).  There is no fallback: if the shared object is missing or fails to
load, every call raises.
"""
import ctypes
import os

import torch  # noqa: F401  (must be imported before the HIP library, see above)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libdpft_ic.so")

ITER_FIRST, ITER_REVERSE, ITER_NO_UPDATE = 0x1, 0x2, 0x4
REMOVE_TRU_SIGMA = 0x1
COMBINE_ICP = 0x2
NO_UNCERTAINTY = 0x4
FEATURES_C4 = 0x8
SCHEDULES = {"auto": 0x00, "march": 0x10, "split": 0x20}  # DPFT_SCHED_*
EXT_SLOT_SHIFT = 12       # DPFT_EXT_SLOT(k) = (k + 1) << 12
EXTREMA_READY = 0x10000
GROUP_SHIFT = 20          # DPFT_GROUP(n) = n << 20: n pairs per independent batch (bits 20-31)
GROUP_MAX_BATCHES = 32
STATUS_NONFINITE = 0x1
CTRL_BYTES = 20480        # the workspace's control area (counters): zero before first use (kCtrlBytes)
ABI_VERSION = 2


class LevelDesc(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int32), ("C", ctypes.c_int32), ("Cs", ctypes.c_int32),
        ("H", ctypes.c_int32), ("W", ctypes.c_int32), ("iters", ctypes.c_int32),
        ("flags", ctypes.c_uint32), ("icp_weight", ctypes.c_float),
    ]


class LevelTensors(ctypes.Structure):
    _fields_ = [
        ("f0", ctypes.c_void_p), ("f1", ctypes.c_void_p), ("s0", ctypes.c_void_p), ("s1", ctypes.c_void_p),
        ("invD0", ctypes.c_void_p), ("invD1", ctypes.c_void_p), ("depth0", ctypes.c_void_p),
        ("depth1", ctypes.c_void_p), ("mask0", ctypes.c_void_p), ("mask1", ctypes.c_void_p),
        ("K", ctypes.c_void_p), ("status", ctypes.c_void_p), ("weights", ctypes.c_void_p),
    ]


EXPORTS = ("dpft_workspace_size", "dpft_ic_solve_level", "dpft_ic_solve_pyramid", "dpft_ic_iterate", "dpft_ic_residual_level",
           "dpft_residual_poses_workspace_size", "dpft_ic_residual_poses", "dpft_ic_residual_map",
           "dpft_ic_reduce_only", "dpft_ic_debug_pixels", "dpft_preprocess_workspace_size",
           "dpft_preprocess_depth", "dpft_pack_features", "dpft_pack_features_nhwc", "dpft_bn_elu", "dpft_bn_elu_pack", "dpft_sigma_extrema_levels", "dpft_ic_damped_update", "dpft_feature_gradient", "dpft_warp_jacobian",
           "dpft_inverse_jacobian", "dpft_normal_equations_workspace_size", "dpft_normal_equations",
           "dpft_read_probe_out_floats", "dpft_read_probe", "dpft_copy_probe", "dpft_version", "dpft_last_error")

_lib = None


def lib():
    """Load (once) and return the CDLL; raises if the native library is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    P = ctypes.POINTER
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.dpft_workspace_size.argtypes = [P(LevelDesc)]
    L.dpft_workspace_size.restype = sz
    L.dpft_ic_solve_level.argtypes = [P(LevelDesc), P(LevelTensors), vp, vp, vp, vp, vp, sz, vp]
    L.dpft_ic_solve_level.restype = ctypes.c_int
    L.dpft_ic_solve_pyramid.argtypes = [P(LevelDesc), P(LevelTensors), ctypes.c_int32, vp, vp, vp, sz, vp]
    L.dpft_ic_solve_pyramid.restype = ctypes.c_int
    L.dpft_ic_iterate.argtypes = [P(LevelDesc), P(LevelTensors), vp, vp, vp, vp, vp, ctypes.c_int, vp, sz, vp]
    L.dpft_ic_iterate.restype = ctypes.c_int
    L.dpft_ic_residual_level.argtypes = [P(LevelDesc), P(LevelTensors), vp, vp, vp, vp, sz, vp]
    L.dpft_ic_residual_level.restype = ctypes.c_int
    L.dpft_residual_poses_workspace_size.argtypes = [P(LevelDesc), ctypes.c_int32]
    L.dpft_residual_poses_workspace_size.restype = sz
    L.dpft_ic_residual_poses.argtypes = [P(LevelDesc), P(LevelTensors), ctypes.c_int32, vp, vp, vp, vp, sz, vp]
    L.dpft_ic_residual_poses.restype = ctypes.c_int
    L.dpft_ic_residual_map.argtypes = [P(LevelDesc), P(LevelTensors), vp, vp, vp, vp, vp, sz, vp]
    L.dpft_ic_residual_map.restype = ctypes.c_int
    L.dpft_ic_reduce_only.argtypes = [P(LevelDesc), P(LevelTensors), vp, vp, vp, sz, vp]
    L.dpft_ic_reduce_only.restype = ctypes.c_int
    L.dpft_ic_debug_pixels.argtypes = [P(LevelDesc), P(LevelTensors), vp, vp, vp, vp, sz, vp]
    L.dpft_ic_debug_pixels.restype = ctypes.c_int
    L.dpft_preprocess_workspace_size.argtypes = []
    L.dpft_preprocess_workspace_size.restype = sz
    L.dpft_preprocess_depth.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                        P(vp), P(vp), vp, sz, vp]
    L.dpft_preprocess_depth.restype = ctypes.c_int
    L.dpft_sigma_extrema_levels.argtypes = [P(LevelDesc), P(LevelTensors), ctypes.c_int32, vp, sz, vp]
    L.dpft_sigma_extrema_levels.restype = ctypes.c_int
    L.dpft_pack_features.argtypes = [vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp]
    L.dpft_pack_features.restype = ctypes.c_int
    L.dpft_pack_features_nhwc.argtypes = [vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp]
    L.dpft_pack_features_nhwc.restype = ctypes.c_int
    L.dpft_bn_elu.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, vp]
    L.dpft_bn_elu.restype = ctypes.c_int
    L.dpft_bn_elu_pack.argtypes = [vp, vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp]
    L.dpft_bn_elu_pack.restype = ctypes.c_int
    L.dpft_ic_damped_update.argtypes = [vp, vp, vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, vp]
    L.dpft_ic_damped_update.restype = ctypes.c_int
    i32 = ctypes.c_int32
    L.dpft_feature_gradient.argtypes = [vp, vp, i32, i32, i32, i32, vp]
    L.dpft_feature_gradient.restype = ctypes.c_int
    L.dpft_warp_jacobian.argtypes = [vp, vp, vp, vp, vp, vp, i32, i32, i32, vp]
    L.dpft_warp_jacobian.restype = ctypes.c_int
    L.dpft_inverse_jacobian.argtypes = [vp] * 8 + [i32] * 5 + [vp]
    L.dpft_inverse_jacobian.restype = ctypes.c_int
    L.dpft_normal_equations_workspace_size.argtypes = [i32]
    L.dpft_normal_equations_workspace_size.restype = sz
    L.dpft_normal_equations.argtypes = [vp, vp, ctypes.c_int64, i32, vp, vp, vp, sz, vp]
    L.dpft_normal_equations.restype = ctypes.c_int
    L.dpft_read_probe_out_floats.argtypes = []
    L.dpft_read_probe_out_floats.restype = sz
    L.dpft_read_probe.argtypes = [vp, sz, ctypes.c_int32, vp, vp]
    L.dpft_read_probe.restype = ctypes.c_int
    L.dpft_copy_probe.argtypes = [vp, vp, sz, ctypes.c_int32, vp]
    L.dpft_copy_probe.restype = ctypes.c_int
    L.dpft_version.argtypes = []
    L.dpft_version.restype = ctypes.c_int
    L.dpft_last_error.argtypes = []
    L.dpft_last_error.restype = ctypes.c_char_p
    if L.dpft_version() != ABI_VERSION:
        raise RuntimeError(f"libdpft_ic ABI {L.dpft_version()} != expected {ABI_VERSION}")
    _lib = L
    return L


def check(rc, what):
    if rc != 0:
        msg = lib().dpft_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")
