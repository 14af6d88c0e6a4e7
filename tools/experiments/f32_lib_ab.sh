#!/bin/bash
# A/B of the default build against libpmm_f32x.so (`make f32x F32X=...`):
# the f32 GPU tests (bit-exact vs the oracle) on both, then c3 and c1
# alternated on the same box
set -o pipefail
mkdir -p gpurun_out
for lib in libpmm.so libpmm_f32x.so; do
  PMM_LIB=$lib timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py -m gpu -k "not bf16" > gpurun_out/fab_tests_$lib.log 2>&1 || exit 2
done
for rep in 1 2; do
  for lib in libpmm_f32x.so libpmm.so; do
    PMM_LIB=$lib timeout -k 10 300 python3 -u bench.py --config c3 --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 0 > gpurun_out/fab_c3_${lib}_$rep.log 2>&1 || exit 3
    PMM_LIB=$lib timeout -k 10 300 python3 -u bench.py --config c1 --steps 200 --warmup 20 --extra none --cpu-sample 0 --boundary 0 --check 0 > gpurun_out/fab_c1_${lib}_$rep.log 2>&1 || exit 4
  done
done
