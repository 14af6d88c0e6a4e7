# wave-specialised bf16 kernel (c4): bf16 parity tests, then ablations
# 0 full, 1 no epilogue, 3 no epilogue + no corpus DMA
mkdir -p gpurun_out
T="true"
timeout -k 10 300 $T > gpurun_out/ws_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/ws_pytest.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --config c4 --steps 3 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 0"
for ab in 0 1 3; do
  timeout -k 10 300 env PMM_ABLATE=$ab $B > gpurun_out/wsab_$ab.json 2>/dev/null || exit 1
  echo "ablate=$ab $(python -c "import json;d=json.load(open('gpurun_out/wsab_$ab.json'));print(d['value'],d['roofline']['achieved'])")"
done
