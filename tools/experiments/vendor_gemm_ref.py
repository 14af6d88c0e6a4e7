"""Reference point for the bf16 roofline fraction: the vendor GEMM (torch.matmul
on ROCm -> hipBLASLt / rocBLAS) on the c4 operand shapes, plain product with
its M x N output and no top-k.  Prints one JSON line per shape.

    python tools/experiments/vendor_gemm_ref.py
"""
import json
import time

import torch

PEAK = {"bf16": 2516.6e12, "f32": 157.3e12}


def bench(m, n, k, dtype, reps=5):
    dev = torch.device("cuda", 0)
    a = torch.randn(m, k, device=dev, dtype=torch.float32).to(dtype)
    b = torch.randn(n, k, device=dev, dtype=torch.float32).to(dtype)
    out = torch.empty(m, n, device=dev, dtype=dtype)
    for _ in range(2):
        torch.matmul(a, b.T, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        torch.matmul(a, b.T, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    fl = 2.0 * m * n * k
    key = "bf16" if dtype == torch.bfloat16 else "f32"
    return {"m": m, "n": n, "k": k, "dtype": key, "ms": round(ms, 3), "tflops": round(fl / ms / 1e9, 1),
            "frac": round(fl / (ms / 1e3) / PEAK[key], 4), "out_bytes": m * n * out.element_size()}


if __name__ == "__main__":
    t0 = time.time()
    for m, n, k, dt in [(100000, 65536, 768, torch.bfloat16), (100000, 16384, 768, torch.bfloat16),
                        (8192, 8192, 8192, torch.bfloat16), (100000, 16384, 768, torch.float32)]:
        print(json.dumps(bench(m, n, k, dt)), flush=True)
    print(json.dumps({"wall_s": round(time.time() - t0, 1), "torch": torch.__version__}))
