#!/bin/bash
# (lab libraries built by: make -C polars-matmul_amd lab LAB="-DPMM_DSX_ABL=<n>" and renamed
#  polars_matmul/libpmm_lab.so -> libpmm_lab_dsx<n>.so / libpmm_lab_sel0.so with LAB="-DPMM_DSX_SEL=0")
# dsx round 2: bf16 dsx tests on the register-select survivor path, then c4
# alternated: ws (default), dsx (shipped), dsx with the LDS re-read (lab
# sel0), dsx pre-filter only (lab abl16, results wrong).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "dsx" --timeout 200 --timeout-method thread \
  > gpurun_out/dsx2_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/dsx2_tests.log
[ $rc -eq 0 ] || exit $rc
B="--config c4 --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0"
run() {  # run <tag> <env...>
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py $B > gpurun_out/dsx2_$tag.json 2> gpurun_out/dsx2_$tag.err || exit 7
  python3 -c "import json;d=json.load(open('gpurun_out/dsx2_$tag.json'));r=d['roofline'];print('$tag', d['ms_per_step'], r['kernel_ms_avg'], r['frac'], r['kernel'][:20], d['check']['exact_index_match_frac'])"
}
for i in 1 2; do
  run ws$i PMM_BF16_DSX=0
  run dsx$i PMM_BF16_DSX=1
  run sel0_$i PMM_BF16_DSX=1 PMM_LIB=libpmm_lab_sel0.so
done
run abl16 PMM_BF16_DSX=1 PMM_LIB=libpmm_lab_dsx16.so
# c1 step time with the per-kernel events on every step vs every 8th / 64th
for st in 1 8 64 1; do
  timeout -k 10 200 python -u bench.py --config c1 --steps 400 --warmup 20 --extra none --cpu-sample 0 --boundary 0 --timing-stride $st \
    > gpurun_out/c1_stride$st.json 2> gpurun_out/c1_stride$st.err || exit 8
  python3 -c "import json;d=json.load(open('gpurun_out/c1_stride$st.json'));r=d['roofline'];print('c1 stride $st', d['ms_per_step'], r['kernel_ms_avg'], r['seed_ms_avg'], r['merge_ms_avg'])"
done
