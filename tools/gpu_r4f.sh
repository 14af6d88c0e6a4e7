#!/bin/bash
# round 4: the whole GPU suite on the current tree (ring seed default, FF
# lab knobs, f64 fused epilogue change), then c1 / c2 / c1_f64 lines and a
# c1 kernel trace (the step's launch timeline)
mkdir -p gpurun_out/r4f
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4f/gpu.log 2>&1
rc=$?
echo "gpu tests rc=$rc"; tail -5 gpurun_out/r4f/gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c1 --steps 2000 --warmup 50 --extra c2,c1_f64,matmul --cpu-sample 0 --boundary 0 > gpurun_out/r4f/c1.json 2> gpurun_out/r4f/c1.log || exit 5
PMC=0 bash tools/profile.sh r4c1 --config c1 --steps 400 --warmup 20 --extra none --cpu-sample 0 --boundary 0 --check 0 || exit 6
echo done
