#!/bin/bash
# k_class_order with wave-level barriers for the short bitonic strides: parity + lines
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu --check 300 --e2e-reps 0"
$S 600 p_tests.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 200 p_c3.json $B &&
$S 200 p_c4.json $B --config 4 &&
$S 200 p_c3_2.json $B
