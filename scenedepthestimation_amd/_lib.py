"""ctypes binding of libsde.so (the C ABI declared in include/sde.h).

torch is imported first on purpose: its bundled HIP runtime (SONAME
libamdhip64.so.7) is then the one libsde.so binds to, so device pointers and
streams handed over from torch are valid in our launches.

There is no fallback: if the library is missing or does not export a symbol of
include/sde.h, importing this module raises.
"""
from __future__ import annotations

import ctypes
import os
import re

import torch  # noqa: F401  (load torch's HIP runtime before libsde.so)

from ._build import INCLUDE, LIB

c_int, c_int64, c_float, c_double, c_void_p = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_double, ctypes.c_void_p
c_char_p = ctypes.c_char_p

SDE_OK = 0
SDE_ABI_VERSION = 4          # include/sde.h: the signatures below are this version's
SDE_LAYOUT_DHW, SDE_LAYOUT_HWD = 0, 1
SDE_WTA_INIT_INF, SDE_WTA_INIT_D0 = 0, 1
SDE_SIDE_LEFT, SDE_SIDE_RIGHT = 1, 2
SDE_TOWER_FP32, SDE_TOWER_BF16X6, SDE_TOWER_F16X3 = 0, 1, 8
SDE_TOWER_IN_CBLOCK, SDE_TOWER_OUT_CBLOCK = 2, 4
SDE_TOWER_WINOGRAD = 16
SDE_TOWER_MFMA32 = 32
SDE_TOWER_IN_SPLIT, SDE_TOWER_OUT_SPLIT = 64, 128
SDE_CV_EXACT, SDE_CV_CERTIFIED = 0, 1
SDE_SGM_ACCUMULATE = 1
SDE_SGM_ZERO_DU_PENALTIES = 2

# name -> (restype, argtypes); must cover every function declared in include/sde.h
SIGNATURES = {
    "sde_abi_version": (c_int, []),
    "sde_status_string": (c_char_p, [c_int]),
    "sde_cost_volume": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_float,
                                c_void_p, c_void_p, c_void_p]),
    "sde_wta": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "sde_cv_wta_workspace_bytes": (c_int64, [c_int, c_int]),
    "sde_cv_wta": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                           c_void_p, c_int, c_void_p, c_int64, c_void_p]),
    "sde_feature_split": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "sde_cv_wta_split_workspace_bytes": (c_int64, [c_int, c_int]),
    "sde_cv_wta_split": (c_int, [c_void_p] * 8 + [c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                                 c_int64, c_void_p]),
    "sde_argmin_merge": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_void_p, c_void_p]),
    "sde_tower_packed_floats": (c_int64, [c_int, c_int]),
    "sde_tower_split_act": (c_int, []),
    "sde_tower_pack_weights": (c_int, [ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p), c_int, c_int,
                                       c_void_p]),
    "sde_tower_workspace_bytes": (c_int64, [c_int, c_int, c_int, c_int]),
    "sde_tower_forward": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                  c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "sde_tower_layer": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p,
                                c_void_p, c_void_p, c_void_p]),
    "sde_tower_batch_workspace_bytes": (c_int64, [c_int, c_int, c_int, c_int, c_int]),
    "sde_tower_forward_batch": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                        c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "sde_tower_layer_scaled": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_int,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "sde_tower_layer_batch": (c_int, [c_void_p, c_int, c_int64, c_int, c_int, c_void_p, c_int, c_int, c_int,
                                      c_void_p, c_int64, c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "sde_absmax_f32": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "sde_set_persistent_grid": (c_int, [c_int]),
    "sde_absmax_f32_batch": (c_int, [c_void_p, c_int, c_int64, c_void_p, c_int, c_void_p]),
    "sde_preprocess_u8_batch": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "sde_preprocess_u8": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "sde_preprocess_scratch_bytes": (c_int64, [c_int, c_int]),
    "sde_sgm_penalties": (c_int, [c_void_p, c_int, c_int, c_double, c_double, c_int64, c_double, c_void_p,
                                  c_void_p]),
    "sde_sgm_8path": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "sde_sgm_8path_pair": (c_int, [c_void_p] * 6 + [c_int, c_int, c_int, c_int, c_void_p]),
    "sde_sgm_8path_wta_pair": (c_int, [c_void_p] * 8 + [c_int, c_int, c_int, c_int, c_void_p]),
    "sde_sgm_direction": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "sde_cbca_arms": (c_int, [c_void_p, c_int64, c_int, c_int, c_int, ctypes.c_float, c_void_p, c_void_p]),
    "sde_cbca_workspace_bytes": (ctypes.c_size_t, [c_int, c_int]),
    "sde_cbca": (c_int, [c_void_p] * 4 + [c_int] * 6 + [c_void_p, ctypes.c_size_t, c_void_p]),
    "sde_cbca_pair": (c_int, [c_void_p] * 6 + [c_int] * 5 + [c_void_p, ctypes.c_size_t, c_void_p]),
    "sde_cbca_lr": (c_int, [c_void_p] * 5 + [c_int] * 5 + [c_void_p, ctypes.c_size_t, c_void_p]),
    "sde_cbca_reciprocals": (c_int, [c_void_p, c_int, c_void_p]),
    "sde_lr_check": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "sde_lrc_fill": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "sde_median5": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
}


def header_functions(path: str = os.path.join(INCLUDE, "sde.h")):
    """Names of the functions declared in include/sde.h (parsed from the header text)."""
    with open(path) as fh:
        text = fh.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sde_[a-z0-9_]+)\s*\(", text)))


class SdeError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB):
        raise ImportError(f"{LIB} is missing: build it with `python -m scenedepthestimation_amd._build` "
                          "(there is no CPU fallback)")
    lib = ctypes.CDLL(LIB)
    missing = []
    for name, (res, args) in SIGNATURES.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            missing.append(name)
            continue
        fn.restype = res
        fn.argtypes = args
    if missing:
        raise ImportError(f"{LIB} does not export {missing}")
    # a library of another ABI would take these argument lists with other meanings (e.g. ABI 3 added
    # the aggregation workspace): refuse it rather than pass it the wrong arguments
    if lib.sde_abi_version() != SDE_ABI_VERSION:
        raise ImportError(f"{LIB} has ABI {lib.sde_abi_version()}, this binding needs {SDE_ABI_VERSION}: rebuild it")
    return lib


lib = _load()


def check(status: int, what: str):
    if status != SDE_OK:
        msg = lib.sde_status_string(status)
        raise SdeError(f"{what} failed: {msg.decode() if msg else status} ({status})")
