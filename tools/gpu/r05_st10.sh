#!/bin/bash
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 r5st_c10.log python -u bench.py --lib karmada_amd/libkp_st10.so --config 10 --steps 2 --warmup 1 --no-cpu --check 0 --inflight 1 --e2e-reps 0
