#!/bin/bash
# A/B on one box: HEAD~ build (libkp_base.so) against the mid-capacity + ranks-in-compact build
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu --check 300 --e2e-reps 0"
$S 600 i_tests.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mid_capacity or test_schedule_parity" &&
$S 200 i_c3_base.json $B --lib karmada_amd/libkp_base.so &&
$S 200 i_c3.json $B &&
$S 200 i_c3_wg.json env KP_TOP_OVER_WG=1 $B &&
$S 200 i_c3_base2.json $B --lib karmada_amd/libkp_base.so &&
$S 200 i_c3_2.json $B &&
$S 200 i_c10_base.json $B --config 10 --lib karmada_amd/libkp_base.so &&
$S 200 i_c10.json $B --config 10 &&
$S 200 i_c5_base.json $B --config 5 --lib karmada_amd/libkp_base.so &&
$S 200 i_c5.json $B --config 5
