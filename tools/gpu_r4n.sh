#!/bin/bash
# round 4: phase removal on the 16x16x32 ws kernel at c4 (lab build;
# PMM_ABLATE: 1 no epilogue, 3 no epilogue and no corpus DMA, 8 pre-filter
# only, 32 hand-off reads only -- results wrong by design)
mkdir -p gpurun_out/r4n
B="--config c4 --steps 2 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 0"
for v in 0 1 3 8 32; do
  PMM_LIB=libpmm_lab.so PMM_ABLATE=$v timeout -k 10 300 python -u bench.py $B > gpurun_out/r4n/abl$v.json 2> gpurun_out/r4n/abl$v.log || { echo "abl $v failed"; exit 5; }
  python3 -c "import json;d=json.load(open('gpurun_out/r4n/abl$v.json'));r=d['roofline'];print('ablate $v', d['ms_per_step'], r['kernel_ms_avg'])"
done
echo done
