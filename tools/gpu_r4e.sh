#!/bin/bash
# round 4: where the fire-and-forget bf16 kernel's time goes at c4 (lab build:
# PMM_ABLATE=1 no pre-filter, =2 pre-filter without stores; PMM_FF_J sets how
# many scores per row pass the guessed threshold), against the shipped ws kernel
mkdir -p gpurun_out/r4e
B="--config c4 --steps 2 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 0"
run() {  # run <name> <env...>
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py $B > gpurun_out/r4e/$name.json 2> gpurun_out/r4e/$name.log || { echo "$name failed"; exit 5; }
  python3 -c "import json;d=json.load(open('gpurun_out/r4e/$name.json'));r=d['roofline'];print('$name', d['ms_per_step'], r['kernel_ms_avg'], r.get('seed_ms_avg'), r.get('merge_ms_avg'))"
}
run ws PMM_LIB=libpmm_lab.so
run ff PMM_LIB=libpmm_lab.so PMM_BF16_FF=1 PMM_FF_DEBUG=1
run ff_abl1 PMM_LIB=libpmm_lab.so PMM_BF16_FF=1 PMM_ABLATE=1
run ff_abl2 PMM_LIB=libpmm_lab.so PMM_BF16_FF=1 PMM_ABLATE=2
run ff_j2 PMM_LIB=libpmm_lab.so PMM_BF16_FF=1 PMM_FF_J=2 PMM_FF_DEBUG=1
run ff_j12 PMM_LIB=libpmm_lab.so PMM_BF16_FF=1 PMM_FF_J=12 PMM_FF_DEBUG=1
echo done
