#!/bin/bash
# ff kernel: its GPU tests, then c4 with and without it (two alternations)
mkdir -p gpurun_out/ff
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "bf16_ff" --timeout 300 --timeout-method thread > gpurun_out/ff/gpu.log 2>&1
rc=$?
echo "ff tests rc=$rc"; tail -3 gpurun_out/ff/gpu.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  PMM_BF16_FF=1 timeout -k 10 300 python -u bench.py --config c4 --steps 5 --warmup 2 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/ff/c4_ff_$i.json 2> gpurun_out/ff/c4_ff_$i.log || exit 5
  timeout -k 10 300 python -u bench.py --config c4 --steps 5 --warmup 2 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/ff/c4_ws_$i.json 2> gpurun_out/ff/c4_ws_$i.log || exit 6
done
# f64 select by ballots: the f64 tests and the c1_f64 line
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "f64 or matmul" --timeout 300 --timeout-method thread > gpurun_out/ff/f64_gpu.log 2>&1 || exit 7
timeout -k 10 300 python -u -c "
import sys, json; sys.argv=['bench.py']
import bench, torch
torch.cuda.set_device(0)
print(json.dumps(bench.f64_line()))
" > gpurun_out/ff/f64_line.json 2> gpurun_out/ff/f64_line.log || exit 8
