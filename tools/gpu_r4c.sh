#!/bin/bash
# probe16 (once), seeding / r64 / set_devices GPU tests, c1/c2 bench lines
mkdir -p gpurun_out/r4c
if [ ! -s gpurun_out/r4b/probe16.txt ]; then
  cd tools/experiments
  for a in 0 1; do
    for m in 1 0 1; do
      timeout -k 10 120 ./bf16_rows64_probe16_a$a 3 $m >> ../../gpurun_out/r4c/probe16.txt 2>&1 || exit 1
    done
  done
  cd ../..
fi
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "seed or r64 or set_devices or pinned or oracle or fixture or kat or ref_" --timeout 400 --timeout-method thread > gpurun_out/r4c/gpu.log 2>&1
rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/r4c/gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c1 --steps 2000 --warmup 50 --extra c2 --cpu-sample 0 --boundary 0 --check 8 > gpurun_out/r4c/c1.json 2> gpurun_out/r4c/c1.log || exit 5
PMM_SEED_MFMA=0 timeout -k 10 300 python -u bench.py --config c1 --steps 2000 --warmup 50 --extra c2 --cpu-sample 0 --boundary 0 --check 8 > gpurun_out/r4c/c1_old.json 2> gpurun_out/r4c/c1_old.log || exit 6
timeout -k 10 300 python -u bench.py --config c1 --steps 2000 --warmup 50 --extra c2 --cpu-sample 0 --boundary 0 --check 8 > gpurun_out/r4c/c1b.json 2> gpurun_out/r4c/c1b.log || exit 7
