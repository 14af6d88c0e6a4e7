#!/bin/bash
# merge kernel at c1 and c3: full, no selection/sort (1), no candidate loads (2)
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 2; do
  PMM_MERGE_ABLATE=$v timeout -k 10 200 python -u bench.py --config c1 --steps 200 --warmup 10 --extra none --cpu-sample 0 --boundary 0 --check 0 > gpurun_out/ma_${v}_c1.log 2>&1 || exit 3
done
