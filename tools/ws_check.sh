# bf16 kernels on the GPU box: parity tests (wave-specialised kernel, then the
# 4-wave kernel), then the c4 bench for each.  Every GPU step time-limited.
mkdir -p gpurun_out
T="python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k bf16"
timeout -k 10 300 $T > gpurun_out/ws_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/ws_pytest.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --config c4 --steps 3 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 8"
timeout -k 10 300 $B > gpurun_out/ws_c4.json 2> gpurun_out/ws_c4.err; rc=$?
echo "ws c4 rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ws_c4.json'));print(d['value'],d['roofline']['achieved'],d.get('check'))")"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 env PMM_BF16_WS=0 $B > gpurun_out/ws0_c4.json 2> gpurun_out/ws0_c4.err; rc=$?
echo "old c4 rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ws0_c4.json'));print(d['value'],d['roofline']['achieved'])")"
exit $rc
