import sys, time, numpy as np
sys.path.insert(0, "polars-matmul_amd")
from polars_matmul import _native
rs = np.random.RandomState(42)
for (m, n, d) in ((1000, 10000, 256), (4000, 50000, 256)):
    q = rs.randn(m, d).astype(np.float32); c = rs.randn(n, d).astype(np.float32)
    for dt in (np.float32, np.float64):
        qq, cc = q.astype(dt), c.astype(dt)
        for _ in range(3): _native.matmul_host(qq, cc)
        t = []
        for _ in range(5):
            t0 = time.perf_counter(); _native.matmul_host(qq, cc); t.append(time.perf_counter() - t0)
        print(m, n, d, dt.__name__, "median ms %.3f" % (1000 * sorted(t)[2]))
