#!/bin/bash
# round 5 baseline: the driver's exact bench command, the 500-step default, config 10
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 r5_drv.json python -u bench.py --gpus 1 --steps 20 --warmup 5 &&
$S 420 r5_def.json python -u bench.py --no-cpu &&
$S 300 r5_c10.json python -u bench.py --config 10 --steps 20 --warmup 2 --no-cpu --check 300 --e2e-reps 0
