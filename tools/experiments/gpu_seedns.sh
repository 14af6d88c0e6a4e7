#!/bin/bash
# c1 step time vs the threshold-seed sample size
set -o pipefail
mkdir -p gpurun_out
for ns in ${NS_LIST:-128 192 256 384}; do
  PMM_SEED_NS=$ns timeout -k 10 200 python -u bench.py --config c1 --steps 200 --warmup 10 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/sn_$ns.log 2>&1 || exit 3
done
