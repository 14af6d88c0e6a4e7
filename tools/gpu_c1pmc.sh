#!/bin/bash
# c1: PMC counters of the merge and the fused kernel
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 -u bench.py --config c1 --steps 20 --warmup 5 --extra none --cpu-sample 0 --boundary 0 --check 0"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/c1pmc_a -o run -- $B > gpurun_out/c1pmc_a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/c1pmc_b -o run -- $B > gpurun_out/c1pmc_b.log 2>&1 || exit 2
