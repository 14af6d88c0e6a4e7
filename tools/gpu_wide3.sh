#!/bin/bash
# 256-row bf16 kernel v2: bf16 parity, c4 bench + ablations
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k bf16 -v -x --timeout 120 --timeout-method thread > gpurun_out/w3_bf16.log 2>&1 || exit 1
B="python3 -u bench.py --config c4 --steps 2 --warmup 1 --extra none --cpu-sample 0 --boundary 0"
for v in "PMM_NONE=0" "PMM_ABLATE=1" "PMM_ABLATE=3"; do
  env $v timeout -k 10 300 $B > gpurun_out/w3_$v.log 2>&1 || exit 2
done
