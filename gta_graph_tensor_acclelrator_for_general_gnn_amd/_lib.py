"""ctypes binding of libgta.so (include/gta.h).

The product path has no fallback: if the HIP library is missing or stale the
import of any op raises.  Build it with `python -c "import __graft_entry__ as g; g.build()"`
or `python -m gta_graph_tensor_acclelrator_for_general_gnn_amd._build`.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgta.so")
ABI_VERSION = 14

# enum mirrors of include/gta.h
GTA_F32, GTA_BF16, GTA_F32_BF16 = 0, 1, 2
DIR_R, DIR_C = 0, 1
IDX_EDGE, IDX_SRC, IDX_DST = 0, 1, 2
OK, ERR_ARG, ERR_HIP, ERR_UNSUPPORTED = 0, -1, -2, -3
BIN_NONE, BIN_ADD, BIN_MUL, BIN_DIV, BIN_SUB = 0, 1, 2, 3, 4
SF = {"NONE": 0, "RELU": 1, "EXP_LEAKY_RELU": 2, "ELU": 3, "EXP": 4, "LEAKY_RELU": 5, "SIGMOID": 6,
      "TANH": 7, "RECIP": 8}

_i64, _i32, _vp, _cp = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p

# name -> (restype, argtypes); every symbol here is declared in include/gta.h
SIGNATURES = {
    "gta_abi_version": (_i32, []),
    "gta_last_error": (_cp, []),
    "gta_scatter": (_i32, [_i32, _vp, _vp, _i64, _i64, _vp, _i64, _i64, _i32, _vp, _i64, _vp]),
    "gta_aggregate": (_i32, [_vp, _vp, _i64, _i64, _i32, _vp, _i64, _i64, _i32, _vp, _i64, _i64, _vp, _vp, _i64,
                             _i32, _vp, _i64, _vp, _vp]),
    "gta_aggregate_self": (_i32, [_vp, _vp, _i64, _i64, _i32, _vp, _i64, _i64, _i32, _vp, _i64, _i64, _vp, _vp, _i64,
                                  _vp, _vp, _i64, _i32, _vp, _i64, _vp, _vp]),
    "gta_aggregate_expr": (_i32, [_vp, _vp, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _i32, _i64, _vp, _i64, _vp,
                                  _i64, _vp, _vp]),
    "gta_aggregate_plan_bytes": (_i64, [_i64, _i64, _i64]),
    "gta_aggregate_plan_build": (_i32, [_vp, _i64, _i64, _i64, _vp, _i64, _vp]),
    "gta_aggregate_workspace_bytes": (_i64, [_i64, _i64, _i64, _i64]),
    "gta_aggregate_blocked_plan_bytes": (_i64, [_i64, _i64, _i64, _i64]),
    "gta_aggregate_blocked_plan_build": (_i32, [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _i64, _vp]),
    "gta_aggregate_blocked_workspace_bytes": (_i64, [_i64, _i64, _i64, _i64, _i64]),
    "gta_aggregate_blocked": (_i32, [_vp, _vp, _i64, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _vp, _i64,
                                     _i32, _vp, _i64, _i64, _vp, _vp]),
    "gta_gat_aggregate_blocked_workspace_bytes": (_i64, [_i64, _i64, _i64, _i64, _i64, _i64]),
    "gta_gat_aggregate_blocked": (_i32, [_vp, _vp, _i64, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _i64, _i32,
                                         _i32, _i32, _vp, _i64, _vp, _vp, _i64, _i64, _vp, _vp]),
    "gta_gather_add": (_i32, [_i32, _vp, _i64, _i64, _vp, _vp, _i64, _vp, _i64, _i64, _vp, _i64, _i32, _vp]),
    "gta_csc_workspace_bytes": (_i64, [_i64, _i64]),
    "gta_csc_build": (_i32, [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _vp]),
    "gta_apply_edge": (_i32, [_i32, _i32, _vp, _vp, _i64, _i64, _vp, _i32, _i64, _i64, _vp, _i32, _i64, _i64, _vp,
                              _i64, _vp]),
    "gta_edge_softmax": (_i32, [_vp, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp]),
    "gta_apply_edge_flat": (_i32, [_i32, _i32, _vp, _vp, _i64, _vp, _i32, _i64, _i64, _vp, _i32, _i64, _i64, _vp, _i64,
                                   _vp]),
    "gta_apply_node": (_i32, [_i32, _i32, _i64, _vp, _i64, _i64, _i32, _vp, _i64, _i64, _vp, _i64, _vp]),
    "gta_update_mm": (_i32, [_vp, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _i32, _i32, _vp, _i64, _vp]),
    "gta_update_mm_t": (_i32, [_vp, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _i32, _i32, _vp, _i64, _vp]),
    "gta_update_mm_t_splits": (_i64, [_i64, _i64, _i64, _i32, _vp]),
    "gta_update_mlp": (_i32, [_vp, _i64, _i64, _i64, _vp, _i64, _i64, _i32, _vp, _i64, _i64, _i32, _i32, _vp, _i64,
                              _vp]),
    "gta_update_mm_t_split_workspace_bytes": (_i64, [_i64, _i64, _i64, _i64]),
    "gta_update_mm_t_split": (_i32, [_vp, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _i32, _i32, _vp, _i64, _i64, _vp,
                                     _i64, _vp]),
    "gta_tile_nnz": (_i32, [_vp, _vp, _i64, _i64, _i64, _vp, _vp]),
    "gta_synth_alpha": (_i32, [_vp, _vp, _i64, _i64, _i32, _i64, _i64, _vp, _vp]),
    "gta_row_ids": (_i32, [_vp, _i64, _i64, _vp, _vp]),
    "gta_build_id": (_cp, []),
    "gta_debug_set": (_i32, [_cp, _i64]),
    "gta_debug_get": (_i32, [_cp, ctypes.POINTER(_i64)]),
    "gta_tuning_create": (_vp, []),
    "gta_tuning_destroy": (None, [_vp]),
    "gta_tuning_set": (_i32, [_vp, _cp, _i64]),
    "gta_tuning_get": (_i32, [_vp, _cp, ctypes.POINTER(_i64)]),
    "gta_tuning_attach": (_i32, [_vp, _vp]),
}

_lock = threading.Lock()
_lib = None


class GTAError(RuntimeError):
    pass


def load(path=LIB_PATH):
    """Load libgta.so and bind every symbol; raises GTAError if anything is missing."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise GTAError(f"libgta.so not found at {path}: the HIP backend is not built "
                           "(run __graft_entry__.build()); there is no CPU fallback")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name, None)
            if fn is None:
                raise GTAError(f"libgta.so lacks symbol {name}")
            fn.restype = res
            fn.argtypes = args
        v = lib.gta_abi_version()
        if v != ABI_VERSION:
            raise GTAError(f"libgta ABI {v} != expected {ABI_VERSION}; rebuild")
        check_build_id(lib.gta_build_id().decode(), path)
        _lib = lib
        return lib


def check_build_id(built, path=LIB_PATH):
    """Refuse a library compiled from other sources than the ones beside it:
    the id is a hash of csrc/gta_kernels.hip + include/gta.h taken at build time (_build.py).
    Where the sources are absent (a library shipped alone) there is nothing to compare against."""
    from . import _build
    want = _build.source_id()
    if want is not None and built != want:
        raise GTAError(f"{path} was built from other sources (build id {built}, sources {want}): "
                       "stale libgta.so -- rebuild with __graft_entry__.build()")


def build_id():
    """The build id of the loaded libgta.so (first 16 hex digits of the sources' sha256)."""
    return load().gta_build_id().decode()


def check(rc, what):
    if rc < 0:
        msg = load().gta_last_error()
        raise GTAError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
    return rc
