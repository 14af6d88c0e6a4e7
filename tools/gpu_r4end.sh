#!/bin/bash
# round 4, last tree: smoke and the default bench line
mkdir -p gpurun_out/r4end
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4end/smoke.log 2>&1 || exit 4
tail -1 gpurun_out/r4end/smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/r4end/bench.json 2> gpurun_out/r4end/bench.log || exit 5
python3 -c "import json;d=json.load(open('gpurun_out/r4end/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac']); e=d['extra']; print('c4', e['c4']['ms_per_step'], e['c4']['roofline']['frac']); print('c1', e['c1']['ms_per_step'], 'c2', e['c2']['ms_per_step'])"
echo done
