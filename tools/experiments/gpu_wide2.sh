#!/bin/bash
# 256-row bf16 kernel ablations at c4 + one PMC pass
set -o pipefail
mkdir -p gpurun_out
B="python3 -u bench.py --config c4 --steps 2 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 0"
for v in "PMM_NONE=0" "PMM_ABLATE=1" "PMM_ABLATE=2" "PMM_ABLATE=3" "PMM_BF16_SYNC=0" "PMM_BF16_WHOLE=0"; do
  env $v timeout -k 10 300 $B > gpurun_out/w2_$v.log 2>&1 || exit 2
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/w2_sq -o run -- $B > gpurun_out/w2_sq.log 2>&1 || exit 3
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/w2_cache -o run -- $B > gpurun_out/w2_cache.log 2>&1 || exit 4
