"""Per-rank shapes of the driver's multi-GPU runs, on one GPU: the c3 and c4
workloads with the corpus cut to 1/2, 1/4 and 1/8 (what each of N ranks
scans: 100k queries x 1M/N rows x 768), the fused kernel's time per launch
against the full corpus's / N.  One JSON line per shape."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "polars-matmul_amd"))
import torch  # noqa: E402

from polars_matmul import _native  # noqa: E402

dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream().cuda_stream
M, N, D, k = 100_000, 1_000_000, 768, 100
g = torch.Generator(device=dev)
g.manual_seed(5)
q = torch.randn((M, D), dtype=torch.float32, device=dev, generator=g)
c = torch.randn((N, D), dtype=torch.float32, device=dev, generator=g)
qb, cb = q.to(torch.bfloat16), c.to(torch.bfloat16)
VARIANTS = json.loads(os.environ.get("SHAPE_VARIANTS", "[]"))  # [[compute, parts, {env}], ...]
cases = [(cp, p, {}) for cp in ("f32", "bf16") for p in (1, 2, 4, 8)] if not VARIANTS else VARIANTS
for compute, parts, env in cases:
    for kk, v in env.items():
        os.environ[kk] = v
    if True:
        n = N // parts
        oi = torch.empty((M, k), dtype=torch.int32, device=dev)
        os_ = torch.empty((M, k), dtype=torch.float32, device=dev)
        if compute == "f32":
            run = lambda: _native.topk_device(q.data_ptr(), D, M, c.data_ptr(), D, n, D, k, 0, oi.data_ptr(),
                                              os_.data_ptr(), stream=stream)
            gname = "gemm_f32_topk"
        else:
            run = lambda: _native.topk_bf16_device(qb.data_ptr(), D, M, cb.data_ptr(), D, n, D, k, 0,
                                                   oi.data_ptr(), os_.data_ptr(), stream=stream)
            gname = "gemm_bf16_topk"
        reps = 2 if compute == "f32" else 4
        run()
        torch.cuda.synchronize()
        _native.timing_reset()
        _native.timing_enable(True)
        t0 = time.perf_counter()
        for _ in range(reps):
            run()
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / reps
        _native.timing_enable(False)
        gms, gn = _native.timing_read(gname)
        tot, _ = _native.timing_read("")
        print(json.dumps({"compute": compute, "M": M, "n": n, "D": D, "k": k, "parts": parts, "env": env,
                          "ms_per_call": round(el * 1000, 3), "kernel_ms": round(gms / max(gn, 1), 3),
                          "all_kernels_ms_per_call": round(tot / reps, 3)}), flush=True)
    for kk in env:
        os.environ.pop(kk)
