#!/bin/bash
# large-slice capacity (LDS per wave -> waves per CU) against fallbacks
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu --check 300 --e2e-reps 0"
$S 200 g_base.json $B &&
$S 200 g_cap512.json env KP_TOP_CAP=512 $B &&
$S 200 g_cap768.json env KP_TOP_CAP=768 $B &&
$S 200 g_cap640.json env KP_TOP_CAP=640 $B
