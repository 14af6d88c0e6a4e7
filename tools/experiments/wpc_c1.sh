#!/bin/bash
# f32 small-problem variant: 1 vs 2 workgroups per CU (PMM_F32_WG_PER_CU) at
# c1 / c2, alternated on one box, plus the f32 GPU tests with 2
set -o pipefail
mkdir -p gpurun_out
PMM_F32_WG_PER_CU=2 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu -k "not bf16" > gpurun_out/wpc_tests.log 2>&1 || exit 2
for rep in 1 2; do
  for w in 1 2; do
    for cfg in c1 c2; do
      PMM_F32_WG_PER_CU=$w timeout -k 10 300 python3 -u bench.py --config $cfg --steps 300 --warmup 30 --extra none --cpu-sample 0 --boundary 0 --check 0 > gpurun_out/wpc_${cfg}_${w}_$rep.log 2>&1 || exit 3
    done
  done
done
