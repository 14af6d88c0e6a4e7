#!/bin/bash
# The 256-row bf16 kernel (lab build: run `make -C polars-matmul_amd lab`
# first): its GPU tests, then c4 with it and with the wave-specialised kernel
# (the shipped default), alternated.
set -o pipefail
mkdir -p gpurun_out
PMM_LIB=libpmm_lab.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "bf16" \
  --timeout 200 --timeout-method thread > gpurun_out/dsx_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/dsx_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 1 0; do
    PMM_LIB=libpmm_lab.so PMM_BF16_DSX=$v timeout -k 10 200 python -u bench.py --config c4 --steps 5 --warmup 2 --extra none \
      --cpu-sample 0 --boundary 0 > gpurun_out/dsx_c4_${v}_${i}.json 2> gpurun_out/dsx_c4_${v}_${i}.err || exit 7
    python3 -c "import json;d=json.load(open('gpurun_out/dsx_c4_${v}_${i}.json'));r=d['roofline'];print('DSX=$v', d['ms_per_step'], r['kernel_ms_avg'], r['frac'], d['check'])"
  done
done
