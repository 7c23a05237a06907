#!/bin/bash
# round 4 final binary: configs 1 and 2 lines
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 c1_final.json python -u bench.py --config 1 --steps 200 --warmup 5 --check 300 --e2e-reps 2 &&
$S 300 c2_final.json python -u bench.py --config 2 --steps 50 --warmup 2 --check 300 --e2e-reps 2
