#!/bin/bash
# round 4: group-granular class-order walk with the hopeless exit (groups of 4; variants 2, 8)
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 i_b3.json python -u bench.py --steps 300 --warmup 5 --no-cpu --check 1000 --e2e-reps 0 &&
$S 300 i_w2.json python -u bench.py --lib karmada_amd/libkp_w2.so --steps 300 --warmup 5 --no-cpu --check 1000 --e2e-reps 0 &&
$S 300 i_w8.json python -u bench.py --lib karmada_amd/libkp_w8.so --steps 300 --warmup 5 --no-cpu --check 1000 --e2e-reps 0 &&
$S 400 i_b5.json python -u bench.py --config 5 --bindings 125000 --steps 20 --warmup 2 --no-cpu --check 500 --e2e-reps 0 &&
$S 600 i_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
