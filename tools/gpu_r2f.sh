#!/bin/bash
# round 2 (resumed): full GPU suite, smoke, default bench, rocprof kernel stats at c3/c4/c1
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 400 --timeout-method thread > gpurun_out/r2f_gpu.log 2>&1
rc1=$?
if [ $rc1 -gt 1 ]; then echo "gpu tests rc=$rc1"; exit $rc1; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2f_smoke.log 2>&1 || exit 4
timeout -k 10 600 python -u bench.py > gpurun_out/r2f_bench.log 2>&1 || exit 5
for cfg in c3 c4 c1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2f_prof_$cfg -o prof -- python3 -u bench.py --config $cfg --steps 5 --warmup 1 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/r2f_prof_$cfg.log 2>&1 || exit 6
done
echo "gpu tests rc=$rc1"
