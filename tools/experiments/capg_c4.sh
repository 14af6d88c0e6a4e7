#!/bin/bash
# c4 step time vs the candidate buffer capacity (PMM_CAPG) with the bf16
# threshold seed on (default): alternated sweep on one box
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for cap in 384 256 320 448 512; do
    PMM_CAPG=$cap timeout -k 10 300 python3 -u bench.py --config c4 --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 0 > gpurun_out/capg_${cap}_$rep.log 2>&1 || exit 3
    echo "capg $cap rep $rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/capg_${cap}_$rep.log)"
  done
done
