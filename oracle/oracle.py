"""ctypes wrapper over the CPU oracle (``libpmm_oracle.so``).

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py``, as the checker or the timed CPU
baseline.  The product package (``polars-matmul_amd/polars_matmul``) never
imports this module.

Every function restates a reference function (paths into the reference tree):

* ``metric_from_str``  -> src/metrics.rs:20-27
* ``norms``            -> src/metrics.rs:368-393
* ``similarity``       -> src/metrics.rs:258-365 (GEMM + epilogue)
* ``select_topk``      -> src/topk.rs:6-75 (the checker's total order, or
                          Rust's select_nth_unstable_by restated for timing)
* ``topk``             -> src/matmul.rs:420-469 (k clipped to N, f32 scores widened to f64)
* ``matmul``           -> src/metrics.rs:40-255 (dst = Q * C^T)
* ``pair_scores``      -> the element S[i, idx[i, j]] of ``similarity`` (f32),
                          without materialising S (full-size parity checks)
* ``topk_blas``        -> src/matmul.rs:420-469 with the reference's STRUCTURE
                          for timing: ndarray-order norms, a threaded BLAS GEMM
                          (OpenBLAS sgemm/dgemm through NumPy in the role of
                          faer's Parallelism::Rayon(0), src/metrics.rs:244-251)
                          into the materialised M x N matrix, then the
                          single-threaded epilogue (:314-365) and per-row
                          select (src/topk.rs:42-75).  The CPU baseline that
                          bench.py times; not the checker (BLAS blocking order
                          differs from the oracle's k-ordered chain).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libpmm_oracle.so")

COSINE, DOT, EUCLIDEAN = 0, 1, 2
_METRIC_NAMES = {COSINE: "cosine", DOT: "dot", EUCLIDEAN: "euclidean"}

_lib = None


def build(force: bool = False) -> str:
    """Compile the oracle with its Makefile (gcc)."""
    if force or not os.path.exists(_LIB_PATH) or (
        os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "pmm_oracle.c"))
    ):
        subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        i64, i32, vp = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p
        L.oracle_metric_from_str.argtypes = [ctypes.c_char_p]
        L.oracle_metric_from_str.restype = i32
        L.oracle_norms_f32.argtypes = [vp, i64, i64, i32, vp]
        L.oracle_norms_f64.argtypes = [vp, i64, i64, i32, vp]
        L.oracle_gemm_f32.argtypes = [vp, i64, vp, i64, i64, vp, i32]
        L.oracle_gemm_f64.argtypes = [vp, i64, vp, i64, i64, vp, i32]
        L.oracle_similarity_f32.argtypes = [vp, i64, vp, i64, i64, i32, vp, i32]
        L.oracle_similarity_f64.argtypes = [vp, i64, vp, i64, i64, i32, vp, i32]
        L.oracle_select_topk_f32.argtypes = [vp, i64, i64, i64, i32, vp, vp]
        L.oracle_select_topk_f64.argtypes = [vp, i64, i64, i64, i32, vp, vp]
        L.oracle_select_topk_rs_f32.argtypes = [vp, i64, i64, i64, i32, vp, vp]
        L.oracle_select_topk_rs_f64.argtypes = [vp, i64, i64, i64, i32, vp, vp]
        L.oracle_topk_f32.argtypes = [vp, i64, vp, i64, i64, i64, i32, i32, vp, vp]
        L.oracle_topk_f32.restype = i64
        L.oracle_topk_f64.argtypes = [vp, i64, vp, i64, i64, i64, i32, i32, vp, vp]
        L.oracle_topk_f64.restype = i64
        L.oracle_pair_scores_f32.argtypes = [vp, i64, vp, i64, i64, i32, vp, i64, i32, vp]
        L.oracle_epilogue_f32.argtypes = [vp, i64, i64, i32, vp, vp]
        L.oracle_epilogue_f64.argtypes = [vp, i64, i64, i32, vp, vp]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def metric_from_str(s: str) -> int:
    """Returns the metric id, or -1 for an unknown name (metrics.rs:20-27)."""
    return lib().oracle_metric_from_str(s.encode())


def _as(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def norms(a: np.ndarray, squared: bool = False) -> np.ndarray:
    a = np.ascontiguousarray(a)
    out = np.empty(a.shape[0], dtype=a.dtype)
    fn = lib().oracle_norms_f32 if a.dtype == np.float32 else lib().oracle_norms_f64
    fn(_p(a), a.shape[0], a.shape[1], int(squared), _p(out))
    return out


def matmul(q: np.ndarray, c: np.ndarray, nthreads: int = 0) -> np.ndarray:
    """dst = Q * C^T in the inputs' dtype (f32 iff both f32, matmul.rs:308)."""
    dt = np.float32 if (q.dtype == np.float32 and c.dtype == np.float32) else np.float64
    q, c = _as(q, dt), _as(c, dt)
    out = np.empty((q.shape[0], c.shape[0]), dtype=dt)
    fn = lib().oracle_gemm_f32 if dt == np.float32 else lib().oracle_gemm_f64
    fn(_p(q), q.shape[0], _p(c), c.shape[0], q.shape[1], _p(out), nthreads)
    return out


def similarity(q: np.ndarray, c: np.ndarray, metric: int, nthreads: int = 0) -> np.ndarray:
    dt = np.float32 if (q.dtype == np.float32 and c.dtype == np.float32) else np.float64
    q, c = _as(q, dt), _as(c, dt)
    out = np.empty((q.shape[0], c.shape[0]), dtype=dt)
    fn = lib().oracle_similarity_f32 if dt == np.float32 else lib().oracle_similarity_f64
    fn(_p(q), q.shape[0], _p(c), c.shape[0], q.shape[1], metric, _p(out), nthreads)
    return out


def select_topk(s: np.ndarray, k: int, higher_is_better: bool, algo: str = "total"):
    """Per-row top-k of a score matrix (src/topk.rs:6-75).  algo="total": the
    checker's quickselect under the fixed total order (score, NaN last, lower
    index); algo="rust": Rust's select_nth_unstable_by + stable sort_by
    restated (pmm_oracle.c, the CPU baseline's select; equal scores in
    whatever order that algorithm leaves them, as in the reference)."""
    s = np.ascontiguousarray(s)
    m, n = s.shape
    idx = np.zeros((m, k), dtype=np.uint32)
    sc = np.zeros((m, k), dtype=s.dtype)
    L = lib()
    if algo == "rust":
        fn = L.oracle_select_topk_rs_f32 if s.dtype == np.float32 else L.oracle_select_topk_rs_f64
    else:
        fn = L.oracle_select_topk_f32 if s.dtype == np.float32 else L.oracle_select_topk_f64
    fn(_p(s), m, n, k, int(higher_is_better), _p(idx), _p(sc))
    return idx, sc


def topk(q: np.ndarray, c: np.ndarray, k: int, metric: int, nthreads: int = 0):
    """(idx uint32 [M,k'], scores float64 [M,k']) with k' = min(k, N)."""
    dt = np.float32 if (q.dtype == np.float32 and c.dtype == np.float32) else np.float64
    q, c = _as(q, dt), _as(c, dt)
    m, d = q.shape
    n = c.shape[0]
    kk = min(k, n)
    idx = np.zeros((m, kk), dtype=np.uint32)
    sc = np.zeros((m, kk), dtype=np.float64)
    fn = lib().oracle_topk_f32 if dt == np.float32 else lib().oracle_topk_f64
    fn(_p(q), m, _p(c), n, d, k, metric, nthreads, _p(idx), _p(sc))
    return idx, sc


def pair_scores(q: np.ndarray, c: np.ndarray, idx: np.ndarray, metric: int, nthreads: int = 0) -> np.ndarray:
    """f32 scores of the (row i, corpus row idx[i, j]) pairs, bit for bit the
    values ``similarity(q, c, metric)[i, idx[i, j]]`` holds (NaN for an empty
    slot, idx 0xFFFFFFFF)."""
    q, c = _as(q, np.float32), _as(c, np.float32)
    idx = np.ascontiguousarray(idx).view(np.uint32) if idx.dtype in (np.int32, np.uint32) else \
        np.ascontiguousarray(idx, dtype=np.uint32)
    m, k = idx.shape
    assert q.shape[0] == m and q.shape[1] == c.shape[1]
    out = np.empty((m, k), dtype=np.float32)
    lib().oracle_pair_scores_f32(_p(q), m, _p(c), c.shape[0], q.shape[1], metric, _p(idx), k,
                                 nthreads, _p(out))
    return out


def topk_blas(q: np.ndarray, c: np.ndarray, k: int, metric: int, nthreads: int = 0, timings: dict = None,
              select: str = "rust"):
    """The reference's topk structure with a BLAS-class threaded GEMM (see the
    module docstring) and, by default, Rust's own select algorithm restated
    (select_topk(algo="rust")).  Returns (idx uint32 [M,k'], scores float64
    [M,k']); `timings`, if given, receives the seconds of each phase (norms,
    gemm, epilogue, select)."""
    import time

    dt = np.float32 if (q.dtype == np.float32 and c.dtype == np.float32) else np.float64
    q, c = _as(q, dt), _as(c, dt)
    m, d = q.shape
    n = c.shape[0]
    kk = min(k, n)
    L = lib()
    t0 = time.perf_counter()
    qn = cn = None
    if metric != DOT:
        qn = norms(q, squared=metric == EUCLIDEAN)
        cn = norms(c, squared=metric == EUCLIDEAN)
    t1 = time.perf_counter()
    if nthreads > 0:
        from threadpoolctl import threadpool_limits

        with threadpool_limits(limits=nthreads, user_api="blas"):
            s = q @ c.T
    else:
        s = q @ c.T
    s = np.ascontiguousarray(s)
    t2 = time.perf_counter()
    if metric != DOT:
        fn = L.oracle_epilogue_f32 if dt == np.float32 else L.oracle_epilogue_f64
        fn(_p(s), m, n, metric, _p(qn), _p(cn))
    t3 = time.perf_counter()
    idx, sc = select_topk(s, kk, metric != EUCLIDEAN, algo=select)
    t4 = time.perf_counter()
    if timings is not None:
        timings.update(norms=t1 - t0, gemm=t2 - t1, epilogue=t3 - t2, select=t4 - t3)
    return idx, sc.astype(np.float64)
