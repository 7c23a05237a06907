#!/bin/bash
# capacity 896 + Webster buffer 192 defaults: parity, config 3/10/5 lines; 5 waves/SIMD variant
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu --check 300 --e2e-reps 0"
$S 600 l_tests.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 200 l_c3.json $B &&
$S 200 l_c3_mw5.json $B --lib karmada_amd/libkp_mw5.so &&
$S 200 l_c3_2.json $B &&
$S 200 l_c10.json $B --config 10 &&
$S 200 l_c5.json $B --config 5 &&
$S 200 l_c4.json $B --config 4
