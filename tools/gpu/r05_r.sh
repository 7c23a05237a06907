#!/bin/bash
# class rows + orders on stream3, k_filter at once on stream2 (KP_ROWS_BESIDE=0: the previous order)
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu --check 300 --e2e-reps 0"
$S 900 r_tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 200 r_c3.json $B &&
$S 200 r_c3_off.json env KP_ROWS_BESIDE=0 $B &&
$S 200 r_c3_2.json $B &&
$S 200 r_c3_off2.json env KP_ROWS_BESIDE=0 $B &&
$S 200 r_c4.json $B --config 4 &&
$S 200 r_c4_off.json env KP_ROWS_BESIDE=0 $B --config 4
