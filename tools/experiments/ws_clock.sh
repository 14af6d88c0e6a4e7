#!/bin/bash
# Cycles or clock?  c4 on the wave-specialised bf16 kernel at PMM_ABLATE=0
# (full), 1 (no epilogue) and 3 (no epilogue, no corpus traffic): kernel
# durations and GRBM_GUI_ACTIVE (effective clock = GUI_ACTIVE / 8 / duration).
# LIBS overrides the library list (e.g. the no-fragment-read diagnostic build
# from `make wsx WSX=-DPMM_WS_NOFRAG`, loaded as libpmm_wsx.so).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/clk
for lib in ${LIBS:-libpmm.so}; do
  for ab in ${ABLATE:-0 1 3}; do
    PMM_LIB=$lib PMM_ABLATE=$ab timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS \
      --output-format csv -d $R/gpurun_out/clk/${lib}_$ab -o run -- python3 $R/bench.py --config c4 --steps 1 --warmup 0 --extra none --cpu-sample 0 --boundary 0 --check 0 \
      > $R/gpurun_out/clk/${lib}_$ab.log 2>&1 || exit 2
  done
done
