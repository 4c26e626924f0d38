"""ctypes binding of oracle/build/liboracle.so (TEST ORACLE / CPU BASELINE ONLY)."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "build/liboracle.so"], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        P, I64, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        for name in ("oracle_aggregate_f32", "oracle_aggregate_heads_f32"):
            f = getattr(lib, name)
            f.restype = None
            f.argtypes = [P, P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I]
        lib.oracle_max_threads.restype = I
        _lib = lib
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def aggregate(indptr, indices, x, w=None, row_begin=0, row_end=None, threads=None):
    """fp32 CSR aggregate over rows [row_begin, row_end) on `threads` host cores."""
    lib = load()
    indptr = np.ascontiguousarray(indptr, dtype=np.int64)
    indices = np.ascontiguousarray(indices, dtype=np.int32)
    x = np.ascontiguousarray(x, dtype=np.float32)
    n = len(indptr) - 1
    row_end = n if row_end is None else row_end
    F = x.shape[1]
    y = np.empty((row_end - row_begin, F), dtype=np.float32)
    threads = threads or lib.oracle_max_threads()
    if w is None:
        lib.oracle_aggregate_f32(_p(indptr), _p(indices), row_begin, row_end, _p(x), F, F, None, 0, 0, _p(y), F,
                                 threads)
    else:
        w = np.ascontiguousarray(w, dtype=np.float32)
        if w.ndim == 1:
            w = w[:, None]
        fn = lib.oracle_aggregate_heads_f32 if F % w.shape[1] == 0 else lib.oracle_aggregate_f32
        fn(_p(indptr), _p(indices), row_begin, row_end, _p(x), F, F, _p(w), w.shape[1], w.shape[1], _p(y), F, threads)
    return y
