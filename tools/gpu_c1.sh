#!/bin/bash
# small-problem path: parity (f32 suite) + c1/c2 latency
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > gpurun_out/c1_parity.log 2>&1 || exit 1
for cfg in c1 c2; do
  timeout -k 10 200 python -u bench.py --config $cfg --steps 200 --warmup 10 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/c1_bench_$cfg.log 2>&1 || exit 3
done
