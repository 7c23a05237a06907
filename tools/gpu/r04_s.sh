#!/bin/bash
# round 4: spread lists grouped by estimator class (vs KP_SPREAD_GROUP=0); GPU suite
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 s_b4.json python -u bench.py --config 4 --steps 50 --warmup 2 --no-cpu --check 300 --e2e-reps 0 &&
$S 300 s_b4_off.json env KP_SPREAD_GROUP=0 python -u bench.py --config 4 --steps 50 --warmup 2 --no-cpu --check 0 --e2e-reps 0 &&
$S 400 s_b5.json python -u bench.py --config 5 --bindings 125000 --steps 20 --warmup 2 --no-cpu --check 300 --e2e-reps 0 &&
$S 600 s_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
