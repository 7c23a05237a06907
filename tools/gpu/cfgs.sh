#!/bin/bash
# Bench lines of the other BASELINE configs (short runs) into gpurun_out/cfg_<n>.log.
mkdir -p gpurun_out
for c in 2 4 6; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 2 --no-cpu --check 300 --e2e-reps 0 > gpurun_out/cfg_$c.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --config 5 --bindings 125000 --steps 5 --warmup 1 --no-cpu --check 300 --e2e-reps 0 > gpurun_out/cfg_5.log 2>&1 || exit $?
for c in 2 4 5 6; do tail -1 gpurun_out/cfg_$c.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print($c, d['ms_per_step'], d['stages_ms'], d['parity_checked'], d['parity_bad'])"; done
