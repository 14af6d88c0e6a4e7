#!/bin/bash
# r64 (PMM_BF16_R64=1) at c4: the full kernel (libpmm_lab.so; it was in the
# shipped libpmm.so when profiles/r3_dsx/r64_ablation.txt was taken) vs lab builds (make -C polars-matmul_amd
# lab LAB=<defines>, renamed libpmm_lab_<name>.so): NOPRE = no pre-filter,
# NOQ = pre-filter without queueing (results wrong), PF2 = two fragments
# ahead, NA6 = six block-1 fragments in AGPRs.
set -o pipefail
mkdir -p gpurun_out
B="--config c4 --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 0"
for lib in libpmm_lab.so libpmm_lab_NOPRE.so libpmm_lab_NOQ.so libpmm_lab_PF2.so libpmm_lab_NA6.so; do
  PMM_BF16_R64=1 PMM_LIB=$lib timeout -k 10 200 python -u bench.py $B > gpurun_out/r64abl_$lib.json 2> gpurun_out/r64abl_$lib.err || exit 7
  python3 -c "import json;d=json.load(open('gpurun_out/r64abl_$lib.json'));r=d['roofline'];print('$lib', d['ms_per_step'], r['kernel_ms_avg'], r['frac'])"
done
