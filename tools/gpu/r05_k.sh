#!/bin/bash
# large-slice LDS: Webster buffer entries (KP_TOP_ECAP) x subset capacity -> workgroups per CU
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu --check 300 --e2e-reps 0"
$S 200 k_cur.json $B &&
$S 200 k_e192.json $B --lib karmada_amd/libkp_ecap192.so &&
$S 200 k_e192_c896.json env KP_TOP_CAP=896 $B --lib karmada_amd/libkp_ecap192.so &&
$S 200 k_e128.json $B --lib karmada_amd/libkp_ecap128.so &&
$S 200 k_e128_c896.json env KP_TOP_CAP=896 $B --lib karmada_amd/libkp_ecap128.so &&
$S 200 k_cur_c896.json env KP_TOP_CAP=896 $B &&
$S 200 k_cur2.json $B
