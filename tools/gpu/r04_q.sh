#!/bin/bash
# round 4: large-subset bindings heaviest first (KP_TOP_LPT=1) vs class-grouped
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 q_lpt.json env KP_TOP_LPT=1 python -u bench.py --steps 300 --warmup 5 --no-cpu --check 1000 --e2e-reps 0 &&
$S 300 q_base.json python -u bench.py --steps 300 --warmup 5 --no-cpu --check 1000 --e2e-reps 0 &&
$S 300 q_lpt2.json env KP_TOP_LPT=1 python -u bench.py --steps 300 --warmup 5 --no-cpu --check 0 --e2e-reps 0
