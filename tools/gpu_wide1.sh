#!/bin/bash
# 256-row bf16 kernel: bf16 parity (all kernels), full-size c4, c4 A/B vs the ws kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k bf16 -v -x --timeout 120 --timeout-method thread > gpurun_out/w1_bf16.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/w1_c4_wide.log 2>&1 || exit 2
PMM_BF16_WIDE=0 timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/w1_c4_ws.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -k c4 -v -s --timeout 400 --timeout-method thread > gpurun_out/w1_full_c4.log 2>&1 || exit 4
