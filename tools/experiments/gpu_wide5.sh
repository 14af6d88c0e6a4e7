#!/bin/bash
# 256-row bf16 kernel: c4 timing + ablations
set -o pipefail
mkdir -p gpurun_out
B="python3 -u bench.py --config c4 --steps 2 --warmup 1 --extra none --cpu-sample 0 --boundary 0"
for v in "PMM_NONE=0" "PMM_ABLATE=1" "PMM_ABLATE=3"; do
  env $v timeout -k 10 300 $B > gpurun_out/w5_$v.log 2>&1 || exit 2
done
