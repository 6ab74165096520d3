#!/bin/bash
# GPU-box job runner: each step under its own time limit; stops at the first
# fatal exit (timeout 124/137, abort 134, segfault 139) so nothing else touches
# a GPU that may be in a bad state.  Ordinary test failures (rc 1) continue.
#   bash scripts/gpu_job.sh TAG "step1-name:seconds:cmd ..." ...
set -u
TAG=$1
shift
mkdir -p gpurun_out
ST=gpurun_out/${TAG}_status.txt
: > "$ST"
for spec in "$@"; do
  name=${spec%%:*}
  rest=${spec#*:}
  tmo=${rest%%:*}
  cmd=${rest#*:}
  echo "[$(date +%T)] $name: $cmd" >> "$ST"
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/${TAG}_${name}.log" 2>&1
  rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> "$ST"
  case $rc in
    124|134|137|139) echo "fatal rc=$rc in $name — stopping" >> "$ST"; cat "$ST"; exit $rc ;;
  esac
done
cat "$ST"
