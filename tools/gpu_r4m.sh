#!/bin/bash
# round 4: per-phase cycle counters of the 16x16x32 ws kernel at c4 (lab
# build with -DPMM_WS_STATS, PMM_STATS=1: wave cycles by role and phase)
mkdir -p gpurun_out/r4m
B="--config c4 --steps 1 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 0"
PMM_LIB=libpmm_stats.so PMM_STATS=1 timeout -k 10 300 python -u bench.py $B > gpurun_out/r4m/stats.json 2> gpurun_out/r4m/stats.log || exit 5
grep "pmm stats" gpurun_out/r4m/stats.log | tail -2
echo done
