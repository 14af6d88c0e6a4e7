#!/bin/bash
# c1/c2 with each f32 tile variant forced (PMM_GEMM_VARIANT)
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 2 3; do
  for cfg in c1 c2; do
    PMM_GEMM_VARIANT=$v timeout -k 10 200 python -u bench.py --config $cfg --steps 200 --warmup 10 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/va_${v}_$cfg.log 2>&1 || exit 3
  done
done
