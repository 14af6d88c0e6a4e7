# rocprofv3 summaries of the current bf16 build at c4 (tools/profile.sh)
bash tools/profile.sh c4fin --config c4 --steps 2 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 0 || exit 1
python tools/pmc_summary.py gpurun_out/prof_c4fin gemm_bf16 > gpurun_out/prof_c4fin/summary.json || exit 1
python tools/pmc_summary.py gpurun_out/prof_c4fin merge_kernel > gpurun_out/prof_c4fin/summary_merge.json || exit 1
