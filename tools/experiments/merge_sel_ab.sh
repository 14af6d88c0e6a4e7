#!/bin/bash
# merge selection over 2/4/8 key slots by candidate count (PMM_MERGE_SEL_E=1,
# default) vs always 8 (lab builds libpmm_lab_sele.so / libpmm_lab_sel8.so,
# plus the shipped libpmm.so): c3 merge time, alternated.
set -o pipefail
mkdir -p gpurun_out
B="--config c3 --steps 2 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 0"
for i in 1 2; do
  for lib in libpmm_lab_sele.so libpmm_lab_sel8.so libpmm.so; do
    PMM_LIB=$lib timeout -k 10 200 python -u bench.py $B > gpurun_out/msel_${lib}_$i.json 2> gpurun_out/msel_${lib}_$i.err || exit 7
    python3 -c "import json;d=json.load(open('gpurun_out/msel_${lib}_$i.json'));r=d['roofline'];m=d['reduction_roofline'];print('$lib', r['merge_ms_avg'], m['frac'])"
  done
done
