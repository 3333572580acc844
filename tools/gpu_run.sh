#!/bin/bash
# Generic GPU-box step runner: bash tools/gpu_run.sh TAG 'cmd1' 'cmd2' ...
# each command runs under its own timeout (first word of the arg if numeric,
# else 300 s), output to gpurun_out/TAG/stepN.log; stops at the first failure.
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
i=0
for c in "$@"; do
  i=$((i+1))
  t=300
  if [[ "$c" =~ ^([0-9]+)\ (.*)$ ]]; then t=${BASH_REMATCH[1]}; c=${BASH_REMATCH[2]}; fi
  echo "== step $i (timeout $t): $c" >> $O/steps.log
  timeout -k 10 $t bash -c "$c" > $O/step$i.log 2>&1
  rc=$?
  echo "   rc=$rc" >> $O/steps.log
  if [ $rc -ne 0 ]; then tail -30 $O/step$i.log; exit $rc; fi
done
echo "all steps ok" >> $O/steps.log
