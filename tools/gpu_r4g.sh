#!/bin/bash
# round 4: f64 tests (fused forced / materialised / default by size), the f64
# lines at c1 and 4096 x 1M x 256, then rocprofv3 summaries of the current
# build at c3, c4 and c1 (kernel trace + the PMC passes of tools/profile.sh)
mkdir -p gpurun_out/r4g
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "f64" --timeout 300 --timeout-method thread > gpurun_out/r4g/gpu_f64.log 2>&1
rc=$?
echo "f64 tests rc=$rc"; tail -3 gpurun_out/r4g/gpu_f64.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --config c1 --steps 200 --warmup 10 --extra c1_f64,f64_large --cpu-sample 0 --boundary 0 --check 0 > gpurun_out/r4g/f64.json 2> gpurun_out/r4g/f64.log || exit 5
bash tools/profile.sh r4_c3 --config c3 --steps 2 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 0 || exit 6
bash tools/profile.sh r4_c4 --config c4 --steps 2 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 0 || exit 7
bash tools/profile.sh r4_c1 --config c1 --steps 200 --warmup 10 --extra none --cpu-sample 0 --boundary 0 --check 0 || exit 8
echo done
