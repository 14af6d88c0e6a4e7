set -o pipefail
A="--steps 2 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 0"
bash tools/profile.sh r2c4b --config c4 $A || exit 1
python tools/pmc_summary.py gpurun_out/prof_r2c4b gemm_bf16 > gpurun_out/prof_r2c4b/summary.json || exit 1
python tools/pmc_summary.py gpurun_out/prof_r2c4b merge_kernel > gpurun_out/prof_r2c4b/summary_merge.json || exit 1
