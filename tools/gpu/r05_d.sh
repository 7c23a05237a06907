#!/bin/bash
# configs 4 / 5 / 10 / 3 lines on the current build
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 r5d_c4.json python -u bench.py --config 4 --steps 100 --warmup 5 --no-cpu --check 500 --e2e-reps 0 &&
$S 400 r5d_c5.json python -u bench.py --config 5 --bindings 125000 --steps 40 --warmup 3 --no-cpu --check 500 --e2e-reps 0 &&
$S 300 r5d_c10.json python -u bench.py --config 10 --steps 40 --warmup 3 --no-cpu --check 500 --e2e-reps 0 &&
$S 300 r5d_c3.json python -u bench.py --steps 200 --warmup 5 --no-cpu --check 500 --e2e-reps 0
