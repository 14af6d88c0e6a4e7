#!/bin/bash
# c1/c2: the 256x256 variant (PMM_GEMM_VARIANT=3) with K order 2 (libpmm.so)
# and 1 (libpmm_korder1.so), against the default choice (128x128, order 1)
set -o pipefail
mkdir -p gpurun_out
for lib in libpmm.so libpmm_korder1.so; do
  for cfg in c1 c2; do
    PMM_LIB=$lib PMM_GEMM_VARIANT=3 timeout -k 10 200 python -u bench.py --config $cfg --steps 200 --warmup 10 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/vk_${lib}_$cfg.log 2>&1 || exit 3
  done
done
for cfg in c1 c2; do
  timeout -k 10 200 python -u bench.py --config $cfg --steps 200 --warmup 10 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/vk_default_$cfg.log 2>&1 || exit 3
done
