#!/bin/bash
# (a "transient" gpurun status means no box or slot was free and nothing ran; any other outcome ends the loop)
# usage: gpu_try.sh OUTFILE TIMEOUT 'command'  -- retries only while no GPU slot/box is free (nothing ran)
out=$1; to=$2; cmd=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out 2>&1
  rc=$?
  if grep -q "status=transient" $out && ! grep -q "status=ok\|status=fail" $out; then sleep 120; continue; fi
  echo "rc=$rc" >> $out; break
done
