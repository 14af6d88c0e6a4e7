# ws kernel: bf16 parity tests (incl. whole-block runs), c4 rate, survivor stats
mkdir -p gpurun_out
T="python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -k bf16"
timeout -k 10 400 $T > gpurun_out/ws_pytest.log 2>&1; rc=$?; grep -E "whole_block|passed|failed|Error" gpurun_out/ws_pytest.log | tail -5; [ $rc -eq 0 ] || exit $rc
B="python bench.py --config c4 --steps 3 --warmup 1 --boundary 0 --extra none --cpu-sample 0"
timeout -k 10 300 $B > gpurun_out/ws_c4.json 2> gpurun_out/ws_c4.err || exit 1
echo "ws c4 $(python -c "import json;d=json.load(open('gpurun_out/ws_c4.json'));print(d['value'],d['roofline']['achieved'],d.get('check'))")"
timeout -k 10 300 env PMM_LIB=libpmm_stats.so PMM_STATS=1 $B --check 0 > gpurun_out/wsst_0.json 2> gpurun_out/wsst_0.err || exit 1
grep 'pmm stats' gpurun_out/wsst_0.err | tail -1
