#!/bin/bash
# round 4: register-resident subsets in k_select_top; k_slow readback only with a region chain
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 420 p_default.json python -u bench.py &&
$S 300 p_b4.json python -u bench.py --config 4 --steps 50 --warmup 2 --no-cpu --check 300 --e2e-reps 0 &&
$S 600 p_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
