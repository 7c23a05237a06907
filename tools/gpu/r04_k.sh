#!/bin/bash
# round 4: k_select_top phase cut-offs (timing only): after the Aggregated cut (x5), after Webster (x4); default bench
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 k_x5.json python -u bench.py --lib karmada_amd/libkp_x5.so --steps 200 --warmup 5 --no-cpu --check 0 --e2e-reps 0 &&
$S 300 k_x4.json python -u bench.py --lib karmada_amd/libkp_x4.so --steps 200 --warmup 5 --no-cpu --check 0 --e2e-reps 0 &&
$S 420 k_default.json python -u bench.py
