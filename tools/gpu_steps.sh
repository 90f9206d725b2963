#!/bin/bash
# Runs GPU steps in order, each under its own time limit, logging to gpurun_out/<name>.log.
#   tools/gpu_steps.sh "name|seconds|command" ...
# An ordinary failure (exit 1, 2, ...) is reported and the next step runs; a time limit (124, 137),
# an abort (134) or a segfault (139) ends the script there, so nothing else touches the GPU after it.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
worst=0
for step in "$@"; do
  name=${step%%|*}; rest=${step#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  case $rc in 124|134|137|139) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
  [ $rc -ne 0 ] && worst=$rc
done
exit $worst
