#!/bin/bash
# round 4: grouped class-order walk in k_select_top (2 chunks per step; variants 4/8, 4/4)
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 g_b3.json python -u bench.py --steps 300 --warmup 5 --no-cpu --check 1000 --e2e-reps 0 &&
$S 300 g_g4.json python -u bench.py --lib karmada_amd/libkp_g4.so --steps 300 --warmup 5 --no-cpu --check 1000 --e2e-reps 0 &&
$S 300 g_g4a4.json python -u bench.py --lib karmada_amd/libkp_g4a4.so --steps 300 --warmup 5 --no-cpu --check 1000 --e2e-reps 0 &&
$S 600 g_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
