#!/bin/bash
# round 4, final tree (resident query rows at c1 / c2): rocprofv3 summaries of
# c1 (kernel trace + PMC passes, for the c1 traffic record), the whole GPU
# suite, smoke and the default bench line
mkdir -p gpurun_out/r4final2
bash tools/profile.sh r4g_c1 --config c1 --steps 200 --warmup 10 --extra none --cpu-sample 0 --boundary 0 --check 0 || exit 8
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4final2/gpu.log 2>&1
rc=$?
echo "gpu tests rc=$rc"; tail -1 gpurun_out/r4final2/gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4final2/smoke.log 2>&1 || exit 4
tail -1 gpurun_out/r4final2/smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/r4final2/bench.json 2> gpurun_out/r4final2/bench.log || exit 5
python3 -c "import json;d=json.load(open('gpurun_out/r4final2/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac']); e=d['extra']; print('c4', e['c4']['ms_per_step'], e['c4']['roofline']['frac'], e['c4']['roofline']['kernel_ms_avg']); print('c1', e['c1']['ms_per_step'], 'c2', e['c2']['ms_per_step']); print('f64_large', {m: e['f64_large'][m]['ms_per_step'] for m in ('fused','materialised','default')})"
echo done
