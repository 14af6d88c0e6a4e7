# candidate-buffer capacity A/B at c4 and c3 (PMM_CAPG), bench only
mkdir -p gpurun_out
for cfg in c4 c3; do
for e in "$@"; do
  timeout -k 10 300 env $e python bench.py --config $cfg --steps 2 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 8 > gpurun_out/cap.json 2> gpurun_out/cap.err || exit 1
  echo "[$cfg $e] $(python -c "import json;d=json.load(open('gpurun_out/cap.json'));print(d['value'],d['roofline']['achieved'],d['roofline']['kernel_ms_avg'],d['check']['valid_topk_frac'],d['reduction_roofline']['kernel_ms_avg'])")"
done
done
