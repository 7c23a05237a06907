#!/bin/bash
# phase stamps (diagnostic build, wrong timings for the line): config 10 and 3
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 r5st_c10.log python -u bench.py --lib karmada_amd/libkp_stamps.so --config 10 --steps 2 --warmup 1 --no-cpu --check 0 --inflight 1 --e2e-reps 0 &&
$S 300 r5st_c3.log python -u bench.py --lib karmada_amd/libkp_stamps.so --config 3 --steps 2 --warmup 1 --no-cpu --check 0 --inflight 1 --e2e-reps 0 &&
$S 300 r5st_pack.log env KP_PACK_TIMING=1 python -u tools/gpu/packtime.py
