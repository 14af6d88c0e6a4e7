#!/bin/bash
# merge_kernel phase costs at c3 (lab build: run `make -C polars-matmul_amd lab`
# first): the shipped library, then the lab library with PMM_MERGE_ABLATE =
# 0 (full), 1 (no final select + sort), 2 (no candidate loads).
set -o pipefail
mkdir -p gpurun_out
B="--config c3 --steps 2 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 0"
run() {  # name lib ablate
  PMM_LIB=$2 PMM_MERGE_ABLATE=$3 timeout -k 10 200 python -u bench.py $B > gpurun_out/mabl_$1.json 2> gpurun_out/mabl_$1.err || exit 7
  python3 -c "import json;d=json.load(open('gpurun_out/mabl_$1.json'));r=d['roofline'];m=d['reduction_roofline'];print('$1', r['merge_ms_avg'], m['frac'], m['bytes_per_launch'])"
}
run shipped libpmm.so 0
run lab0 libpmm_lab.so 0
run lab1 libpmm_lab.so 1
run lab2 libpmm_lab.so 2
run lab0b libpmm_lab.so 0
