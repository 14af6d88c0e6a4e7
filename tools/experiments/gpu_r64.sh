#!/bin/bash
# One-wave-per-SIMD 256-row bf16 kernel (PMM_BF16_R64; lab build: run `make -C
# polars-matmul_amd lab` first): its GPU tests (bit equality with the
# wave-specialised kernel), then c4 alternated r64 / ws.
export PMM_LIB=libpmm_lab.so
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "r64 or d128" --timeout 200 --timeout-method thread \
  > gpurun_out/r64_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r64_tests.log
[ $rc -eq 0 ] || exit $rc
B="--config c4 --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0"
for i in 1 2; do
  for v in 1 0; do
    PMM_BF16_R64=$v timeout -k 10 200 python -u bench.py $B > gpurun_out/r64_c4_${v}_$i.json 2> gpurun_out/r64_c4_${v}_$i.err || exit 7
    python3 -c "import json;d=json.load(open('gpurun_out/r64_c4_${v}_$i.json'));r=d['roofline'];print('R64=$v', d['ms_per_step'], r['kernel_ms_avg'], r['seed_ms_avg'], r['frac'], r['kernel'][:22], d['check']['exact_index_match_frac'])"
  done
done
