#!/bin/bash
# Tuning experiments on the GPU box: each line = one bench run of a library variant.
# usage: bash exp.sh "<label> <lib> <env...>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  set -- $spec
  label=$1; lib=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --lib karmada_amd/libkp_$lib.so --steps 50 --warmup 2 --no-cpu --check 0 > gpurun_out/exp_$label.log 2>&1
  rc=$?
  python3 -c "
import json,sys
try:
  d=json.loads(open('gpurun_out/exp_$label.log').read().strip().split('\n')[-1])
  print('$label', d['ms_per_step'], d['stages_ms'])
except Exception as e: print('$label', 'rc=$rc', e)
"
  if [ $rc -gt 1 ]; then exit $rc; fi
done
