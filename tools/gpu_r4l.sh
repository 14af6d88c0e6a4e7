#!/bin/bash
# round 4: the 16x16x32 ws kernel's compile-time epilogue knobs at c4, lab
# builds alternated twice (def / NST=6 ring slots / survivor drain every 2
# tiles / epilogue column groups 1 interval apart)
mkdir -p gpurun_out/r4l
B="--config c4 --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 0"
for i in 1 2; do
  for v in def nst6 dr2 sp1; do
    PMM_LIB=libpmm_ab_$v.so timeout -k 10 300 python -u bench.py $B > gpurun_out/r4l/${v}_$i.json 2> gpurun_out/r4l/${v}_$i.log || { echo "$v failed"; exit 5; }
    python3 -c "import json;d=json.load(open('gpurun_out/r4l/${v}_$i.json'));r=d['roofline'];print('$v $i', d['ms_per_step'], r['kernel_ms_avg'], r['frac'])"
  done
done
echo done
