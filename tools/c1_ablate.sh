# f32 kernel at c1 / c2 (the reference's benchmark size): full, filter only
# (ablate=2), no epilogue (ablate=1)
mkdir -p gpurun_out
for cfg in c1 c2; do
for e in PMM_ABLATE=0 PMM_ABLATE=2 PMM_ABLATE=1; do
  timeout -k 10 300 env $e python bench.py --config $cfg --steps 20 --warmup 3 --boundary 0 --extra none --cpu-sample 0 --check 0 > gpurun_out/c1a.json 2> gpurun_out/c1a.err || exit 1
  echo "[$cfg $e] $(python -c "import json;d=json.load(open('gpurun_out/c1a.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms_avg'],d['roofline']['merge_ms_avg'])")"
done
done
