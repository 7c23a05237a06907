#!/bin/bash
# round 4: Webster phase stamps in k_select_top (config 3)
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 l_stamps3.log env KP_TOP_SPLIT=0 python -u bench.py --lib karmada_amd/libkp_stamps.so --steps 2 --warmup 1 --no-cpu --check 0 --inflight 1 --e2e-reps 0
