#!/bin/bash
# GPU suite, then config 3/4/5 bench lines (parity re-checked) on this build
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 900 r5b_gputest.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread &&
$S 300 r5b_c4.json python -u bench.py --config 4 --steps 100 --warmup 5 --no-cpu --check 500 --e2e-reps 0 &&
$S 400 r5b_c5.json python -u bench.py --config 5 --bindings 125000 --steps 40 --warmup 3 --no-cpu --check 500 --e2e-reps 0 &&
$S 300 r5b_c3.json python -u bench.py --steps 200 --warmup 5 --no-cpu --check 500 --e2e-reps 2
