#!/bin/bash
# step.sh <seconds> <log> <cmd...>: one GPU step under its own time limit; rc 0/1
# (passed / a test or parity failure) lets the caller go on, anything else (a fault,
# an abort, a time limit) ends the whole GPU command with that code.
t=$1; log=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1
rc=$?
echo "[step] $log rc=$rc" >> gpurun_out/steps.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
exit 0
