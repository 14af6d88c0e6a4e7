set -e
mkdir -p gpurun_out
B="python bench.py --config c4 --steps 3 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 4"
for v in 1 0 1 0; do
  env PMM_BF16_DEFER=$v timeout -k 10 300 $B > gpurun_out/ab_defer_$v.json 2>gpurun_out/ab_defer_err.log
  echo "defer=$v $(python -c "import json;d=json.load(open('gpurun_out/ab_defer_$v.json'));print(d['value'],d['roofline']['achieved'])")"
done
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k bf16 > gpurun_out/ab_defer_pytest.log 2>&1 && tail -3 gpurun_out/ab_defer_pytest.log
