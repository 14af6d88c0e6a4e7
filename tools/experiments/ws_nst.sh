#!/bin/bash
# wave-specialised bf16 kernel: c4 with the current ring depth (+ no-epilogue ablation)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k bf16 -q -x --timeout 120 --timeout-method thread > gpurun_out/nst_bf16.log 2>&1 || exit 1
for v in PMM_NONE=0 PMM_ABLATE=1; do
  env $v timeout -k 10 300 python3 -u bench.py --config c4 --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/nst_$v.log 2>&1 || exit 2
done
