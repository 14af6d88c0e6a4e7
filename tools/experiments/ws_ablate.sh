# bf16 ws kernel at c4: full, no epilogue (ablate=1), no corpus traffic and no
# epilogue (ablate=3); TFLOP/s each.  Every GPU step time-limited.
mkdir -p gpurun_out
B="python bench.py --config c4 --steps 2 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 0"
for ab in 0 1 3; do
  timeout -k 10 300 env PMM_ABLATE=$ab $B > gpurun_out/wsab_$ab.json 2> gpurun_out/wsab_$ab.err || exit 1
  echo "ablate=$ab $(python -c "import json;d=json.load(open('gpurun_out/wsab_$ab.json'));print(d['value'],d['roofline']['achieved'],d['roofline']['kernel_ms_avg'])")"
done
