#!/bin/bash
# Run GPU steps in order, each under its own time limit; a step that fails normally (rc 1, e.g. a
# failing test) lets the next run, anything else (fault, abort, segfault, timeout) ends the call.
# usage: tools/gpu_steps.sh "<seconds> <log> <cmd...>" ...
for step in "$@"; do
  read -r secs log cmd <<<"$step"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "step [$cmd] rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
