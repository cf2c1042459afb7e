#!/bin/bash
# Run named GPU steps, each under its own time limit, logging to gpurun_out/<name>.log.
# Stops the session on any crash-class exit (fault/abort/segv/timeout); plain
# failures (exit 1/2/5, e.g. failing asserts) continue to the next step.
#   tools/gpu_session.sh <name> <timeout_s> <cmd...> [-- <name> <timeout_s> <cmd...>]...
mkdir -p gpurun_out
export TMPDIR=/tmp
while [ $# -gt 0 ]; do
  name=$1; t=$2; shift 2
  cmd=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do cmd+=("$1"); shift; done
  [ "$1" == "--" ] && shift
  echo "== $name (limit ${t}s): ${cmd[*]}"
  start=$(date +%s)
  timeout -k 10 "$t" "${cmd[@]}" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "rc=$rc ($(( $(date +%s) - start ))s)"
  tail -n 15 "gpurun_out/$name.log"
  case $rc in
    0|1|2|5) ;;
    *) echo "FATAL rc=$rc in step $name: stopping session"; exit $rc ;;
  esac
done
exit 0
