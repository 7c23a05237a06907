#!/bin/bash
# k_select_top large slice at capacity 512 first, overflow relaunch at 1024: parity + lines
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu --check 300 --e2e-reps 0"
$S 600 h_tests.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mid_capacity or top_histogram or test_schedule_parity" &&
$S 200 h_c3.json $B &&
$S 200 h_c3_nomid.json env KP_TOP_CAP_MID=0 $B &&
$S 200 h_c10.json $B --config 10 &&
$S 200 h_c5.json $B --config 5
