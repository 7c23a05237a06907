#!/bin/bash
# A/B on one box: 16-bit subset ranks (+ ranks mapped in k_compact) against HEAD~; mid capacities
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu --check 300 --e2e-reps 0"
$S 600 j_tests.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mid_capacity or test_schedule_parity" &&
$S 200 j_c3_base.json $B --lib karmada_amd/libkp_base.so &&
$S 200 j_c3.json $B &&
$S 200 j_c3_mid512.json env KP_TOP_CAP_MID=512 $B &&
$S 200 j_c3_mid768.json env KP_TOP_CAP_MID=768 $B &&
$S 200 j_c3_base2.json $B --lib karmada_amd/libkp_base.so &&
$S 200 j_c3_2.json $B &&
$S 200 j_c10_base.json $B --config 10 --lib karmada_amd/libkp_base.so &&
$S 200 j_c10.json $B --config 10
