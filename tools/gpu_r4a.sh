#!/bin/bash
# round 4, first check: -m gpu suite, smoke, default bench line (new legs)
set -o pipefail
mkdir -p gpurun_out/r4a
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/r4a/gpu.log 2>&1
rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/r4a/gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a/smoke.log 2>&1 || exit 4
timeout -k 10 900 python -u bench.py > gpurun_out/r4a/bench.json 2> gpurun_out/r4a/bench.log || exit 5
PMM_BENCH_INPROC_DEVICES=0,0 timeout -k 10 300 python -u bench.py --inproc-child 2 --config c3 --steps 3 --warmup 1 > gpurun_out/r4a/inproc.json 2> gpurun_out/r4a/inproc.log || exit 6
exit $rc
