# c1 seed-pass cost breakdown: kernel trace under PMM_ABLATE=0 (full),
# 2 (filter only), 1 (no epilogue); seed and main launches alternate
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $root/gpurun_out
cd /tmp && export TMPDIR=/tmp
for ab in 0 2 1; do
  PMM_ABLATE=$ab timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $root/gpurun_out/sabl_$ab -o run -- python3 $root/bench.py --config c1 --steps 30 --warmup 3 --boundary 0 --extra none --cpu-sample 0 --check 0 > $root/gpurun_out/sabl_$ab.log 2>&1 || exit 1
  python3 - $root/gpurun_out/sabl_$ab/run_kernel_trace.csv $ab <<'PY'
import csv,sys
tr=list(csv.DictReader(open(sys.argv[1])))
g=[int(t['End_Timestamp'])-int(t['Start_Timestamp']) for t in tr if 'gemm_f32' in t['Kernel_Name']]
m=[int(t['End_Timestamp'])-int(t['Start_Timestamp']) for t in tr if 'merge_kernel' in t['Kernel_Name']]
print('ablate',sys.argv[2],'gemm seed/main us',sum(g[0::2])/len(g[0::2])/1e3,sum(g[1::2])/len(g[1::2])/1e3,'merge',sum(m[0::2])/len(m[0::2])/1e3,sum(m[1::2])/len(m[1::2])/1e3)
PY
done
