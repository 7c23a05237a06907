#!/bin/bash
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 r5c_c10.json python -u bench.py --config 10 --steps 40 --warmup 3 --no-cpu --check 300 --e2e-reps 0
