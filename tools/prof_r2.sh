#!/bin/bash
# round-2 rocprofv3 summaries of the current build: c3 (f32 headline), c4
# (bf16), c1 (the reference's benchmark size): kernel trace + stats, then the
# PMC passes (tools/profile.sh) and their summaries (tools/pmc_summary.py).
set -o pipefail
A="--steps 2 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 0"
bash tools/profile.sh r2c3 --config c3 $A || exit 1
python tools/pmc_summary.py gpurun_out/prof_r2c3 gemm_f32 > gpurun_out/prof_r2c3/summary.json || exit 1
python tools/pmc_summary.py gpurun_out/prof_r2c3 merge_kernel > gpurun_out/prof_r2c3/summary_merge.json || exit 1
bash tools/profile.sh r2c4 --config c4 $A || exit 1
python tools/pmc_summary.py gpurun_out/prof_r2c4 gemm_bf16 > gpurun_out/prof_r2c4/summary.json || exit 1
python tools/pmc_summary.py gpurun_out/prof_r2c4 merge_kernel > gpurun_out/prof_r2c4/summary_merge.json || exit 1
PMC=0 bash tools/profile.sh r2c1 --config c1 --steps 50 --warmup 5 --boundary 0 --extra none --cpu-sample 0 --check 0 || exit 1
