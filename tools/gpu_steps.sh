#!/bin/bash
# Run GPU steps in order, each "<seconds> <command...>" line from stdin under its own time limit;
# a pytest step that only has failing tests (rc 1) does not stop the chain, anything else non-zero
# (fault, abort, timeout) does. usage: tools/gpu_steps.sh < steps.txt
set -u
while IFS= read -r line; do
  [ -z "$line" ] && continue
  lim=${line%% *}; cmd=${line#* }
  echo "== $cmd"
  timeout -k 10 "$lim" bash -c "$cmd"
  rc=$?
  if [ $rc -ne 0 ]; then
    case "$cmd" in *pytest*|*gpu_tests.sh*) [ $rc -eq 1 ] && { echo "(tests failed, rc 1: continuing)"; continue; };; esac
    echo "step failed rc=$rc: stopping"; exit $rc
  fi
done
