# bf16 (c4) per-phase statistics and ablations on the GPU box.
mkdir -p gpurun_out
B="python bench.py --config c4 --steps 2 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 0"
timeout -k 10 300 env PMM_STATS=1 $B > gpurun_out/c4_stats.json 2> gpurun_out/c4_stats.err || exit 1
grep "pmm stats" gpurun_out/c4_stats.err | tail -2
for ab in 0 1 2; do
  timeout -k 10 300 env PMM_ABLATE=$ab $B > gpurun_out/c4_ab$ab.json 2>/dev/null || exit 1
  echo "ablate=$ab $(python -c "import json;d=json.load(open('gpurun_out/c4_ab$ab.json'));print(d['value'],d['roofline']['achieved'])")"
done
