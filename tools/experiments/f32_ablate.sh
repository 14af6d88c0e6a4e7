# f32 kernel at c3: full, filter pass only (ablate=2), no epilogue (ablate=1)
mkdir -p gpurun_out
for e in PMM_ABLATE=0 PMM_ABLATE=2 PMM_ABLATE=1; do
  timeout -k 10 300 env $e python bench.py --config c3 --steps 2 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 0 > gpurun_out/fa.json 2> gpurun_out/fa.err || exit 1
  echo "[$e] $(python -c "import json;d=json.load(open('gpurun_out/fa.json'));print(d['value'],d['roofline']['achieved'],d['roofline']['kernel_ms_avg'])")"
done
