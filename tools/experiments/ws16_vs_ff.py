"""The 16x16x32 form of the wave-specialised bf16 kernel (PMM_WS_MFMA16,
loaded as PMM_LIB=libpmm_ws16.so) against the fire-and-forget kernel, which
runs the same v_mfma_f32_16x16x32_bf16 chain per 16 x 16 block in natural K
order: the two lists must agree bit for bit (indices and f32 scores)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "polars-matmul_amd"))
from polars_matmul import _native as n  # noqa: E402

M = {"cosine": 0, "dot": 1, "euclidean": 2}
bad = 0
for (m, nn, d, k) in [(300, 70000, 256, 10), (520, 200000, 768, 100), (257, 131072, 384, 32),
                      (1000, 100003, 128, 20), (70, 90000, 640, 8), (4096, 300000, 768, 100)]:
    rs = np.random.RandomState(m + nn + d + k)
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(nn, d).astype(np.float32)
    c[nn // 2:nn // 2 + 20] = c[:20]
    for metric in ("cosine", "dot", "euclidean"):
        os.environ["PMM_BF16_FF"] = "0"
        wi, wsc = n.topk_host(q, c, k, M[metric], compute=n.COMPUTE_BF16)
        os.environ["PMM_BF16_FF"] = "1"
        fi, fsc = n.topk_host(q, c, k, M[metric], compute=n.COMPUTE_BF16)
        same_i = np.array_equal(wi, fi)
        same_s = np.array_equal(wsc.view(np.uint64), fsc.view(np.uint64))
        print(f"{m}x{nn}x{d} k={k} {metric}: indices equal {same_i}, scores equal {same_s}, "
              f"index agreement {np.mean(wi == fi):.6f}", flush=True)
        bad += (not same_i) + (not same_s)
print("ws16 == ff" if bad == 0 else f"{bad} mismatches")
sys.exit(1 if bad else 0)
