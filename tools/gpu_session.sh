#!/bin/bash
# Run a sequence of GPU steps on the gpurun box, each under its own time limit; stop at the
# first fault-like exit (timeout, abort, segfault, signal).  Logs go to gpurun_out/<name>.log.
#   tools/gpu_session.sh "name|timeout_s|command" ...
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
export TMPDIR=${TMPDIR:-/tmp}
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; to=${rest%%|*}; cmd=${rest#*|}
  echo "=== [$name] (limit ${to}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "$OUT/$name.log"
  case $rc in
    0|1) ;;                      # success / test failures: keep going
    *) echo "=== fatal exit $rc in [$name]: stopping"; exit $rc ;;
  esac
done
