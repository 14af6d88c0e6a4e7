#!/bin/bash
# A/B of the default build against libpmm_wsx.so (`make wsx WSX=...`) at c4,
# in one call (box-to-box clock differences exceed most effects): bf16
# parity tests on both, then the c4 bench alternated B, A, B, A
set -o pipefail
mkdir -p gpurun_out
for lib in libpmm.so libpmm_wsx.so; do
  PMM_LIB=$lib timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py -m gpu -k "bf16" > gpurun_out/lab_tests_$lib.log 2>&1 || exit 2
done
for rep in 1 2; do
  for lib in libpmm_wsx.so libpmm.so; do
    PMM_LIB=$lib timeout -k 10 300 python3 -u bench.py --config c4 --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 0 > gpurun_out/lab_${lib}_$rep.log 2>&1 || exit 3
  done
done
