#!/bin/bash
# Merge scratch layout A/B (PMM_MERGE_SWZ: shipped = 2 XOR swizzle; lab
# builds libpmm_lab_swz0.so = plain, libpmm_lab_swz1.so = padded, made by
# make -C polars-matmul_amd lab LAB=-DPMM_MERGE_SWZ=<n> and renamed): the merge
# and multi-device GPU tests on the shipped build, then c3 and c1 alternated.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/swz_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/swz_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for lib in libpmm.so libpmm_lab_swz0.so libpmm_lab_swz1.so; do
    for cfg in c3 c1; do
      st=2; [ $cfg = c1 ] && st=400
      PMM_LIB=$lib timeout -k 10 200 python -u bench.py --config $cfg --steps $st --warmup 2 --extra none --cpu-sample 0 --boundary 0 \
        > gpurun_out/swz_${lib}_${cfg}_$i.json 2> gpurun_out/swz_${lib}_${cfg}_$i.err || exit 7
      python3 -c "import json;d=json.load(open('gpurun_out/swz_${lib}_${cfg}_$i.json'));r=d['roofline'];print('$lib $cfg', d['ms_per_step'], r['kernel_ms_avg'], r['merge_ms_avg'], d['reduction_roofline']['frac'], d['check']['exact_index_match_frac'])"
    done
  done
done
