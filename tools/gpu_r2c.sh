#!/bin/bash
# round 2: bit-exact parity, c3 A/B of the K-order builds, full-size parity, smoke
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v --maxfail=20 --timeout 120 --timeout-method thread > gpurun_out/r2c_parity.log 2>&1
rc1=$?
if [ $rc1 -gt 1 ]; then exit $rc1; fi
for lib in libpmm.so libpmm_korder0.so libpmm_korder1.so; do
  PMM_LIB=$lib timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/r2c_bench_$lib.log 2>&1 || exit 3
done
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2c_smoke.log 2>&1 || exit 4
timeout -k 10 700 python -u -m pytest tests/test_gpu_fullsize.py -v -s --timeout 400 --timeout-method thread > gpurun_out/r2c_fullsize.log 2>&1
rc2=$?
echo "parity rc=$rc1 fullsize rc=$rc2"
