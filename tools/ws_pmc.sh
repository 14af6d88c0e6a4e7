# clock and LDS counters of the bf16 ws kernel under ablations (one pmc pass each)
mkdir -p gpurun_out/wspmc
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for ab in 0 1 3; do
  PMM_ABLATE=$ab timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/wspmc/ab$ab -o run -- python3 $R/bench.py --config c4 --steps 2 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 0 > $R/gpurun_out/wspmc/ab$ab.log 2>&1 || exit 1
  echo "ablate=$ab done"
done
