set -o pipefail
CFGS="c1 c2 c3" bash tools/gpu_lib_ab.sh libpmm_prev.so libpmm.so || exit 1
cp gpurun_out/lib_ab.txt gpurun_out/lib_ab_split.txt
for rep in 1 2; do
  for v in 0 4; do
    for cfg in c1 c2; do
      PMM_GEMM_VARIANT=$v timeout -k 10 120 python -u bench.py --config $cfg --steps 400 --warmup 20 --extra none --cpu-sample 0 --boundary 0 --check 8 > gpurun_out/v4.json 2>/dev/null || exit 2
      python -c "import json,sys; d=json.loads(open('gpurun_out/v4.json').read().strip().splitlines()[-1]); r=d['roofline']; print('variant', $v, '$cfg', 'step', d['ms_per_step'], 'gemm', r['kernel_ms_avg'], 'merge', r['merge_ms_avg'], 'exact', d['check']['exact_index_match_frac'])" >> gpurun_out/v4_ab.txt
    done
  done
done
cat gpurun_out/v4_ab.txt
PMM_GEMM_VARIANT=4 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parity_v4.log 2>&1; echo parity_v4 rc=$?; tail -2 gpurun_out/parity_v4.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parity_split2.log 2>&1; echo parity rc=$?; tail -2 gpurun_out/parity_split2.log
