#!/bin/bash
# Run one GPU step with its own time limit; classify the outcome so a caller chain can stop after
# any GPU fault:  exit 0 = ok, 1 = test failures only, 99 = fault / abort / timeout (stop the chain).
# usage: scripts/gpustep.sh <seconds> <logfile> <command...>
secs=$1; log=$2; shift 2
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
if grep -q -E "illegal memory access|Memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|GPU Hang|core dumped" "$log"; then
  echo "[gpustep] GPU fault signature in $log (rc=$rc)"; exit 99
fi
case $rc in
  0) exit 0 ;;
  1) exit 1 ;;
  *) echo "[gpustep] abnormal exit rc=$rc ($log)"; exit 99 ;;
esac
