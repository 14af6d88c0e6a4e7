#!/bin/bash
# rocprofv3 summaries of the current build for c3 (f32 headline) and c1 (the
# reference's benchmark size): tools/profile.sh passes + tools/pmc_summary.py
set -o pipefail
A="--steps 2 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 0"
bash tools/profile.sh r2c3b --config c3 $A || exit 1
python tools/pmc_summary.py gpurun_out/prof_r2c3b gemm_f32 > gpurun_out/prof_r2c3b/summary.json || exit 1
python tools/pmc_summary.py gpurun_out/prof_r2c3b merge_kernel > gpurun_out/prof_r2c3b/summary_merge.json || exit 1
PMC=0 bash tools/profile.sh r2c1b --config c1 --steps 50 --warmup 5 --boundary 0 --extra none --cpu-sample 0 --check 0 || exit 1
