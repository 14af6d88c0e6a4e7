"""f64 top-k, fused scan vs materialised scores, by problem size (device
API, inputs resident, cosine): where the size rule of pmm_capi.hip
(f64_fused_enabled) should put its threshold.  One JSON line per size."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "polars-matmul_amd"))

import torch  # noqa: E402

from polars_matmul import _native  # noqa: E402

SIZES = [(1000, 10_000, 256, 10), (1000, 100_000, 256, 10), (4096, 100_000, 256, 10),
         (1000, 1_000_000, 256, 10), (4096, 1_000_000, 256, 10), (4096, 1_000_000, 256, 100),
         (4096, 1_000_000, 256, 1)]
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream().cuda_stream
for M, N, D, k in SIZES:
    g = torch.Generator(device=dev)
    g.manual_seed(M + N)
    q = torch.randn((M, D), dtype=torch.float64, device=dev, generator=g)
    c = torch.randn((N, D), dtype=torch.float64, device=dev, generator=g)
    oi = torch.empty((M, k), dtype=torch.int32, device=dev)
    os_ = torch.empty((M, k), dtype=torch.float64, device=dev)
    rec = {"M": M, "N": N, "D": D, "k": k, "matrix_gb": round(M * N * 8 / 1e9, 3)}
    outs = {}
    for mode in ("1", "0"):
        os.environ["PMM_F64_FUSED"] = mode
        reps = 20 if M * N <= 1e8 else 3
        for _ in range(2):
            _native.topk_f64_device(q.data_ptr(), D, M, c.data_ptr(), D, N, D, k, 0, oi.data_ptr(), os_.data_ptr(),
                                    stream=stream)
        torch.cuda.synchronize()
        _native.timing_reset()
        _native.timing_enable(True)
        t0 = time.perf_counter()
        for _ in range(reps):
            _native.topk_f64_device(q.data_ptr(), D, M, c.data_ptr(), D, N, D, k, 0, oi.data_ptr(), os_.data_ptr(),
                                    stream=stream)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / reps
        _native.timing_enable(False)
        name = "fused" if mode == "1" else "materialised"
        rec[name + "_ms"] = round(el * 1000, 3)
        rec[name + "_fell_back"] = _native.timing_read("gemm_f64_scores")[1] > 0 if mode == "1" else None
        rec[name + "_gemm_launches"] = (_native.timing_read("gemm_f64_topk" if mode == "1" else "gemm_f64_scores")[1]
                                        // reps)
        outs[name] = (oi.clone(), os_.clone())
    os.environ.pop("PMM_F64_FUSED")
    rec["same_lists"] = bool(torch.equal(outs["fused"][0], outs["materialised"][0]) and
                             torch.equal(outs["fused"][1], outs["materialised"][1]))
    print(json.dumps(rec), flush=True)
    del q, c
    torch.cuda.empty_cache()
