#!/bin/bash
# round 4: k_select_top phase cut-offs (timing only): after the walk (x2), after sel_all_fast's sums (x3)
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 j_x2.json python -u bench.py --lib karmada_amd/libkp_x2.so --steps 200 --warmup 5 --no-cpu --check 0 --e2e-reps 0 &&
$S 300 j_x3.json python -u bench.py --lib karmada_amd/libkp_x3.so --steps 200 --warmup 5 --no-cpu --check 0 --e2e-reps 0 &&
$S 300 j_b3.json python -u bench.py --steps 200 --warmup 5 --no-cpu --check 0 --e2e-reps 0
