#!/bin/bash
# round 4: k_select_top small-slice threshold (replicas + spec.Clusters), 100 / 160 / 230
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 r_n100.json env KP_TOP_SMALL_NEED=100 python -u bench.py --steps 300 --warmup 5 --no-cpu --check 1000 --e2e-reps 0 &&
$S 300 r_n230.json env KP_TOP_SMALL_NEED=230 python -u bench.py --steps 300 --warmup 5 --no-cpu --check 1000 --e2e-reps 0 &&
$S 300 r_n160.json python -u bench.py --steps 300 --warmup 5 --no-cpu --check 0 --e2e-reps 0
