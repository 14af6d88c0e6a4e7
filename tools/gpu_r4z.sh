#!/bin/bash
# round 4: f32 small variants -- resident query rows (AK) and the LDS survivor
# queue: full GPU suite, c1 / c2 A/B of both (alternated twice), a kernel
# trace of c1 / c2, then the default bench line
mkdir -p gpurun_out/r4z
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4z/gpu.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r4z/gpu.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, AK, QCAP
PMM_F32_AK=$2 PMM_F32_QCAP=$3 timeout -k 10 300 python -u bench.py --config c1 --steps 1000 --warmup 50 --extra c2 --cpu-sample 0 --boundary 0 --check 8 > gpurun_out/r4z/c1_$1.json 2> gpurun_out/r4z/c1_$1.log || exit 5
python3 -c "import json;d=json.load(open('gpurun_out/r4z/c1_$1.json'));r=d['roofline'];print('$1 c1', d['ms_per_step'], r.get('kernel_ms_avg'), 'c2', d['extra']['c2']['ms_per_step'], d['extra']['c2']['roofline'].get('kernel_ms_avg'), 'exact', d['check']['exact_index_match_frac'])"
}
for rep in 1 2; do run ak1q1 1 1; run ak1q0 1 0; run ak0q1 0 1; run ak0q0 0 0; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4z/prof -o run -- python3 bench.py --config c1 --steps 300 --warmup 20 --extra c2 --cpu-sample 0 --boundary 0 --check 0 > gpurun_out/r4z/prof.log 2>&1 || exit 6
find gpurun_out/r4z/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r4z/kernel_stats.csv \;
timeout -k 10 600 python -u bench.py > gpurun_out/r4z/bench.json 2> gpurun_out/r4z/bench.log || exit 7
python3 -c "import json;d=json.load(open('gpurun_out/r4z/bench.json'));e=d['extra'];print(d['value'], d['ms_per_step'], d['roofline']['frac'], 'c4', e['c4']['ms_per_step'], e['c4']['roofline']['frac'], 'c1', e['c1']['ms_per_step'], 'c2', e['c2']['ms_per_step'])"
echo done
