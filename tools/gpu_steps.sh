#!/bin/bash
# Run GPU steps in order, each "NAME|SECONDS|COMMAND"; output of step NAME goes to
# gpurun_out/NAME.log.  A step that fails on its own (e.g. a red test) does not stop the
# rest; a time limit (124 / 137), an abort (134) or a segfault (139) ends the script there.
#   gpurun -- 'bash tools/gpu_steps.sh "a|300|python -u x.py" "b|200|python -u y.py"'
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -4 "gpurun_out/$name.log"
  case $rc in 124|137|134|139) echo "fatal rc $rc: stopping"; exit $rc;; esac
done
