# bf16 ws kernel A/B at c4: each argument is an env setting (e.g.
# "PMM_BF16_PM=2 PMM_ABLATE=16"); for each, the bf16 parity tests then the c4
# bench.  Every GPU step time-limited; stops at the first failure.
mkdir -p gpurun_out
B="python bench.py --config c4 --steps 3 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 8"
i=0
for e in "$@"; do
  i=$((i+1))
  timeout -k 10 300 env $e python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k bf16 > gpurun_out/ws_pytest_$i.log 2>&1; rc=$?
  echo "[$e] pytest rc=$rc $(tail -1 gpurun_out/ws_pytest_$i.log)"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 env $e $B > gpurun_out/wsab_$i.json 2> gpurun_out/wsab_$i.err || exit 1
  echo "[$e] $(python -c "import json;d=json.load(open('gpurun_out/wsab_$i.json'));print(d['value'],d['roofline']['achieved'],d['roofline']['kernel_ms_avg'],d['check']['valid_topk_frac'])")"
done
