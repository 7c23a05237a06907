#!/bin/bash
# k_class_order on stream3 beside k_filter (component-set rows first): full GPU suite + lines
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu --check 300 --e2e-reps 0"
$S 900 q_tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 200 q_c3.json $B &&
$S 200 q_c4.json $B --config 4 &&
$S 300 q_c5.json $B --config 5 &&
$S 200 q_c3_2.json $B
