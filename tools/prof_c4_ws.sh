# rocprofv3 summaries of the current bf16 (wave-specialised) kernel at c4:
# kernel trace + stats, then the PMC passes (tools/profile.sh)
bash tools/profile.sh c4ws --config c4 --steps 2 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 0 || exit 1
python tools/pmc_summary.py gpurun_out/prof_c4ws gemm_bf16 > gpurun_out/prof_c4ws/summary.json
cat gpurun_out/prof_c4ws/summary.json
