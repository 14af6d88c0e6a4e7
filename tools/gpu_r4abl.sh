#!/bin/bash
# round 4: c1 / c2 epilogue split on the final tree (lab build, PMM_ABLATE:
# 0 full, 2 pre-filter without survivor handling, 1 no epilogue), alternated twice
mkdir -p gpurun_out/r4abl
for rep in 1 2; do for ab in 0 2 1; do
PMM_LIB=libpmm_lab.so PMM_ABLATE=$ab timeout -k 10 300 python -u bench.py --config c1 --steps 1000 --warmup 50 --extra c2 --cpu-sample 0 --boundary 0 --check 0 > gpurun_out/r4abl/c1_$ab.json 2> gpurun_out/r4abl/c1_$ab.log || exit 5
python3 -c "import json;d=json.load(open('gpurun_out/r4abl/c1_$ab.json'));r=d['roofline'];c=d['extra']['c2'];print('ablate $ab c1 step', d['ms_per_step'], 'fused', r.get('kernel_ms_avg'), '| c2 step', c['ms_per_step'], 'fused', c['roofline'].get('kernel_ms_avg'))"
done; done
echo done
