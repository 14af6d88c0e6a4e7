# rocprofv3 summaries of the current build: c3 (f32 headline) and c4 (bf16),
# kernel trace + stats, then the PMC passes (tools/profile.sh); summaries.
set -o pipefail
bash tools/profile.sh c3fin --config c3 --steps 2 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 0 || exit 1
python tools/pmc_summary.py gpurun_out/prof_c3fin gemm_f32 > gpurun_out/prof_c3fin/summary.json || exit 1
python tools/pmc_summary.py gpurun_out/prof_c3fin merge_kernel > gpurun_out/prof_c3fin/summary_merge.json || exit 1
bash tools/profile.sh c4fin --config c4 --steps 2 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 0 || exit 1
python tools/pmc_summary.py gpurun_out/prof_c4fin gemm_bf16 > gpurun_out/prof_c4fin/summary.json || exit 1
python tools/pmc_summary.py gpurun_out/prof_c4fin merge_kernel > gpurun_out/prof_c4fin/summary_merge.json || exit 1
grep -h '"avg_ms"\|mfma_busy\|hbm_bytes_per_launch\|effective_clock' gpurun_out/prof_c3fin/summary.json gpurun_out/prof_c4fin/summary.json
