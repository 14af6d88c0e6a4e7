#!/bin/bash
# round 2: bit-exact parity (natural K order by 4-byte LDS-DMA gathers, correctly
# rounded sqrt), full-size parity, c3 A/B of the K-order variants
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v --maxfail=20 --timeout 120 --timeout-method thread > gpurun_out/r2b_parity.log 2>&1
rc1=$?
if [ $rc1 -gt 1 ]; then exit $rc1; fi
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/r2b_bench_k2.log 2>&1 || exit 3
PMM_LIB=libpmm_korder0.so timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/r2b_bench_k0.log 2>&1 || exit 4
timeout -k 10 700 python -u -m pytest tests/test_gpu_fullsize.py -v -s --timeout 400 --timeout-method thread > gpurun_out/r2b_fullsize.log 2>&1
rc2=$?
echo "parity rc=$rc1 fullsize rc=$rc2"
