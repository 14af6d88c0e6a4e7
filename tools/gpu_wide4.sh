#!/bin/bash
# 256-row bf16 kernel v2: failure pattern of the bf16 tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k bf16 -q --timeout 120 --timeout-method thread > gpurun_out/w4_bf16.log 2>&1
echo rc=$?
