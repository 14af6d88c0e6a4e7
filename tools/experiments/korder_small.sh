#!/bin/bash
# c1/c2 latency of the f32 K-order builds (Makefile korder target):
# libpmm.so (4-byte DMA gathers), libpmm_korder1.so (16-byte DMA + permlane
# swaps), libpmm_korder3.so (query image by 16-byte DMA + swaps)
set -o pipefail
mkdir -p gpurun_out
for lib in libpmm.so libpmm_korder1.so libpmm_korder3.so; do
  for cfg in c1 c2; do
    PMM_LIB=$lib timeout -k 10 200 python -u bench.py --config $cfg --steps 200 --warmup 10 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/ko_${lib}_$cfg.log 2>&1 || exit 3
  done
done
