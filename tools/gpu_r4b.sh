#!/bin/bash
# 16x16x32 rows64 probe (both data modes), then the r64 cross-check and
# set_devices tests through the lab binding in the default suite
mkdir -p gpurun_out/r4b
cd tools/experiments
for a in 0 1; do
  for m in 1 0 1; do
    timeout -k 10 120 ./bf16_rows64_probe16_a$a 3 $m >> ../../gpurun_out/r4b/probe16.txt 2>&1 || exit 1
  done
done
cd ../..
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "r64 or set_devices or pinned" --timeout 400 --timeout-method thread > gpurun_out/r4b/gpu.log 2>&1
rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/r4b/gpu.log
exit $rc
