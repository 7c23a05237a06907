#!/bin/bash
# one Cp-bit mask for the walk and the target bits (-640 B per wave); 8 workgroups per CU
# needs <= 10 240 B per wave: capacity x Webster buffer combinations
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu --check 300 --e2e-reps 0"
$S 600 n_tests.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 200 n_c3.json $B &&
$S 200 n_c3_c768.json env KP_TOP_CAP=768 $B &&
$S 200 n_c3_e128.json $B --lib karmada_amd/libkp_e128.so &&
$S 200 n_c3_e160_c832.json env KP_TOP_CAP=832 $B --lib karmada_amd/libkp_e160.so &&
$S 200 n_c3_2.json $B &&
$S 200 n_c10.json $B --config 10 &&
$S 200 n_c10_e128.json $B --config 10 --lib karmada_amd/libkp_e128.so
