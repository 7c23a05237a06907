#!/bin/bash
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu --check 300 --e2e-reps 0"
$S 200 h_c3.json $B --lib karmada_amd/libkp_hoist2.so &&
$S 200 h_c10.json $B --config 10 --lib karmada_amd/libkp_hoist2.so &&
$S 200 h_c3base.json $B
