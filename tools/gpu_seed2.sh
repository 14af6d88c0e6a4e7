#!/bin/bash
# one-launch threshold seeding: parity + c1/c2 latency
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > gpurun_out/s2_parity.log 2>&1 || exit 1
for cfg in c1 c2; do
  timeout -k 10 200 python -u bench.py --config $cfg --steps 200 --warmup 10 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/s2_bench_$cfg.log 2>&1 || exit 3
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s2_prof_c1 -o run -- python3 -u bench.py --config c1 --steps 50 --warmup 5 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/s2_prof_c1.log 2>&1 || exit 4
