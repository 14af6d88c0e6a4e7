#!/bin/bash
# round 2, first GPU pass: MFMA order probe, bit-exact parity, full-size parity, c3 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/mfma_order_probe > gpurun_out/r2_probe.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v --maxfail=30 --timeout 120 --timeout-method thread > gpurun_out/r2_parity.log 2>&1
rc1=$?
if [ $rc1 -gt 1 ]; then exit $rc1; fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -v -s -x --timeout 400 --timeout-method thread > gpurun_out/r2_fullsize.log 2>&1
rc2=$?
if [ $rc2 -gt 1 ]; then exit $rc2; fi
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/r2_bench_nat.log 2>&1 || exit 3
PMM_LIB=libpmm_kperm.so timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/r2_bench_kperm.log 2>&1 || exit 4
echo "parity rc=$rc1 fullsize rc=$rc2"
