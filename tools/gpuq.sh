#!/bin/bash
# usage: gpuq.sh <outfile> <timeout> <command>   -- re-submits only while no box is free (rc 3 / transient)
# (run from this container: tools/gpuq.sh /tmp/x.out 1200 "bash tools/gpu_x.sh")
out=$1; to=$2; shift 2
for i in $(seq 1 15); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1
  rc=$?
  if grep -q "no free box\|stopped responding while being prepared\|backing off\|taken away\|slot(s) on this pod are busy" $out && ! grep -q "status=ok\|status=fail" $out; then sleep 100; continue; fi
  exit $rc
done
exit $rc
