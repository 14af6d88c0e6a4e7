"""f64 top-k (the path Polars' default Float64 columns take) at the reference
benchmark's size: host call time, f64 vs f32."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "polars-matmul_amd"))
from polars_matmul import _native as n  # noqa: E402

np.random.seed(42)
q = np.random.randn(1000, 256)
c = np.random.randn(10000, 256)
for dt in (np.float32, np.float64):
    qq, cc = q.astype(dt), c.astype(dt)
    for _ in range(3):
        n.topk_host(qq, cc, 10, 0)
    ts = []
    for _ in range(20):
        t0 = time.perf_counter()
        n.topk_host(qq, cc, 10, 0)
        ts.append(time.perf_counter() - t0)
    print(dt.__name__, "%.3f ms" % (np.median(ts) * 1e3))
n.timing_reset()
n.timing_enable(True)
for _ in range(10):
    n.topk_host(q, c, 10, 0)
n.timing_enable(False)
for name in ("gemm_f64_scores", "merge_chunks", "norms_f64", "norms_"):
    print(name, n.timing_read(name))
