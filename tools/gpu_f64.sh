#!/bin/bash
# f64 path: GPU tests (-k f64 / matmul) and the c1_f64 bench line
set -o pipefail
mkdir -p gpurun_out/f64
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "f64 or matmul or ref_" --timeout 300 --timeout-method thread > gpurun_out/f64/gpu.log 2>&1
rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/f64/gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "
import sys, json; sys.argv=['bench.py']
import bench, torch
torch.cuda.set_device(0)
print(json.dumps(bench.f64_line()))
" > gpurun_out/f64/line.json 2> gpurun_out/f64/line.log || exit 5
exit $rc
