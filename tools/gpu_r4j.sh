#!/bin/bash
# round 4: the whole GPU suite with the 16x16x32 wave-specialised kernel as the
# default (ws == ff bit-exact cross-checks), smoke, then the default bench
mkdir -p gpurun_out/r4j
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4j/gpu.log 2>&1
rc=$?
echo "gpu tests rc=$rc"; tail -5 gpurun_out/r4j/gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4j/smoke.log 2>&1 || exit 4
tail -1 gpurun_out/r4j/smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/r4j/bench.json 2> gpurun_out/r4j/bench.log || exit 5
python3 -c "import json;d=json.load(open('gpurun_out/r4j/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac']); e=d['extra']; print('c4', e['c4']['ms_per_step'], e['c4']['roofline']['frac'], e['c4']['roofline']['kernel_ms_avg']); print('c1', e['c1']['ms_per_step'], 'c2', e['c2']['ms_per_step'])"
echo done
