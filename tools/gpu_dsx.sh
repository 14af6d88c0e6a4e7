#!/bin/bash
# bf16 256-row kernel check: the bf16 GPU tests (both kernels), then c4 with
# the new kernel and with the wave-specialised one, alternated.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "bf16" --timeout 200 --timeout-method thread \
  > gpurun_out/dsx_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/dsx_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 1 0; do
    PMM_BF16_DSX=$v timeout -k 10 200 python -u bench.py --config c4 --steps 5 --warmup 2 --extra none --cpu-sample 0 --boundary 0 \
      > gpurun_out/dsx_c4_${v}_${i}.json 2> gpurun_out/dsx_c4_${v}_${i}.err || exit 7
    python3 -c "import json;d=json.load(open('gpurun_out/dsx_c4_${v}_${i}.json'));r=d['roofline'];print('DSX=$v', d['ms_per_step'], r['kernel_ms_avg'], r['frac'], d['check'])"
  done
done
