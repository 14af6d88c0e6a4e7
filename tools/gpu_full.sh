#!/bin/bash
# full check: -m gpu suite, smoke, default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > gpurun_out/full_gpu.log 2>&1
rc=$?
echo "gpu tests rc=$rc"; tail -2 gpurun_out/full_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 || exit 4
timeout -k 10 600 python -u bench.py > gpurun_out/full_bench.log 2>&1 || exit 5
exit $rc
