# wave-specialised bf16 kernel (c4): epilogue-wave phase cycles (diagnostics
# build) for the PMM_ABLATE values given as arguments
mkdir -p gpurun_out
B="python bench.py --config c4 --steps 2 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 0"
for ab in "$@"; do
  timeout -k 10 300 env PMM_LIB=libpmm_stats.so PMM_STATS=1 PMM_ABLATE=$ab $B > gpurun_out/wsst_$ab.json 2> gpurun_out/wsst_$ab.err || exit 1
  echo "stats-build ablate=$ab $(python -c "import json;d=json.load(open('gpurun_out/wsst_$ab.json'));print(d['value'],d['roofline']['achieved'])") $(grep 'pmm stats' gpurun_out/wsst_$ab.err | tail -1)"
done
