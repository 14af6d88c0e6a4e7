#!/bin/bash
# round 2: parity (seeding, chunked upload), c1/c2 latency, c3 with host-boundary rates
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v --maxfail=10 --timeout 120 --timeout-method thread > gpurun_out/r2e_parity.log 2>&1
rc1=$?
if [ $rc1 -gt 1 ]; then exit $rc1; fi
for cfg in c1 c2; do
  timeout -k 10 200 python -u bench.py --config $cfg --steps 200 --warmup 10 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/r2e_bench_$cfg.log 2>&1 || exit 3
done
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 1 > gpurun_out/r2e_bench_c3.log 2>&1 || exit 4
echo "parity rc=$rc1"
