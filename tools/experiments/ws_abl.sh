# bf16 ws kernel at c4, bench only (no tests): each argument is an env setting
mkdir -p gpurun_out
B="python bench.py --config c4 --steps 3 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 0"
i=0
for e in "$@"; do
  i=$((i+1))
  timeout -k 10 300 env $e $B > gpurun_out/wsabl_$i.json 2> gpurun_out/wsabl_$i.err || exit 1
  echo "[$e] $(python -c "import json;d=json.load(open('gpurun_out/wsabl_$i.json'));print(d['value'],d['roofline']['achieved'],d['roofline']['kernel_ms_avg'])")"
done
