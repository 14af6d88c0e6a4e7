#!/bin/bash
# c3 A/B of f32 kernel builds on one box: PMM_LIB=<lib> bench.py (3 steps each)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > gpurun_out/ab_parity.log 2>&1 || exit 1
for lib in "$@"; do
  PMM_LIB=$lib timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/ab_$lib.log 2>&1 || exit 3
done
