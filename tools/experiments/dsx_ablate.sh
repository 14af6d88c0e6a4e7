#!/bin/bash
# (lab libraries built by: make -C polars-matmul_amd lab LAB="-DPMM_DSX_ABL=<n>" and renamed
#  polars_matmul/libpmm_lab.so -> libpmm_lab_dsx<n>.so / libpmm_lab_sel0.so with LAB="-DPMM_DSX_SEL=0")
# bf16 256-row kernel (dsx) diagnosis at c4: lab ablation builds (compile-time
# PMM_DSX_ABL: 1 no epilogue, 2 no corpus DMA, 4 no MFMAs, 8 no fragment
# reads), then the rocprofv3 passes of tools/profile.sh on the shipped build,
# then the FETCH_SIZE calibration program.
set -o pipefail
mkdir -p gpurun_out
B="--config c4 --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0"
for lib in libpmm.so libpmm_lab_dsx1.so libpmm_lab_dsx3.so libpmm_lab_dsx5.so libpmm_lab_dsx7.so libpmm_lab_dsx9.so; do
  PMM_LIB=$lib timeout -k 10 200 python -u bench.py $B > gpurun_out/abl_$lib.json 2> gpurun_out/abl_$lib.err || exit 7
  python3 -c "import json;d=json.load(open('gpurun_out/abl_$lib.json'));r=d['roofline'];print('$lib', d['ms_per_step'], r['kernel_ms_avg'], r['seed_ms_avg'], r['frac'])"
done
bash tools/profile.sh r3c4dsx $B --check 0 || exit 8
python tools/pmc_summary.py gpurun_out/prof_r3c4dsx gemm_bf16_dsx > gpurun_out/prof_r3c4dsx/summary.json || exit 9
cat gpurun_out/prof_r3c4dsx/summary.json
bash tools/calib/run_calib.sh || exit 10
