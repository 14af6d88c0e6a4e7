#!/bin/bash
# round 4: XCD-grouped tile order for the f64 GEMM tile (store + fused scan):
# f64 tests, then the size sweep (fused vs materialised)
mkdir -p gpurun_out/r4r
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "f64 or matmul" --timeout 300 --timeout-method thread > gpurun_out/r4r/gpu_f64.log 2>&1
rc=$?; echo "f64 tests rc=$rc"; tail -3 gpurun_out/r4r/gpu_f64.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/experiments/f64_sizes.py > gpurun_out/r4r/f64_sizes.jsonl 2> gpurun_out/r4r/f64_sizes.log || exit 5
cat gpurun_out/r4r/f64_sizes.jsonl
echo done
