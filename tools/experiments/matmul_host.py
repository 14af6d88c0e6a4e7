"""`.pmm.matmul` host path at the c1 size: where the per-call time goes
(fresh vs reused output buffer; the output D2H vs the input uploads)."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "polars-matmul_amd"))
from polars_matmul import _native as n  # noqa: E402

np.random.seed(42)
q = np.random.randn(1000, 256).astype(np.float32)
c = np.random.randn(10000, 256).astype(np.float32)
lib = n._lib
ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731


def t(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return np.median(ts) * 1e3


out = np.empty((1000, 10000), np.float32)
out.fill(0)
print("fresh output  %.3f ms" % t(lambda: n.matmul_host(q, c)))
print("reused output %.3f ms" % t(lambda: lib.pmm_matmul_f32(ptr(q), 1000, ptr(c), 10000, 256, ptr(out))))
small = np.empty((1000, 10), np.float32)
print("1000x10 out   %.3f ms" % t(lambda: lib.pmm_matmul_f32(ptr(q), 1000, ptr(c[:10]), 10, 256, ptr(small))))
print("np.empty+fill %.3f ms" % t(lambda: np.empty((1000, 10000), np.float32).fill(0)))
