#!/bin/bash
# k_select_top occupancy experiments (config 3, 100 steps each)
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu --check 200 --e2e-reps 0"
$S 200 occ_base.json $B &&
$S 200 occ_mw5.json $B --lib karmada_amd/libkp_mw5.so &&
$S 200 occ_mw6.json $B --lib karmada_amd/libkp_mw6.so &&
KP_TOP_CAP=512 $S 200 occ_cap512.json $B &&
KP_TOP_CAP=512 $S 200 occ_mw5_cap512.json $B --lib karmada_amd/libkp_mw5.so
