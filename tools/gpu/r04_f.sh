#!/bin/bash
# round 4: k_slow on workgroup-scope barriers, cheaper stop rule: config 8 seed 6 passes,
# GPU suite, config 3/5 lines, the walk's ring depth (8, 12 chunks ahead)
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 f_diag8.log python -u tools/gpu/diag_cfg8.py karmada_amd/libkp.so 8:6:300:1500 20 &&
$S 600 f_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 300 f_b3.json python -u bench.py --steps 300 --warmup 5 --no-cpu --check 1000 --e2e-reps 3 &&
$S 300 f_a8.json python -u bench.py --lib karmada_amd/libkp_a8.so --steps 200 --warmup 3 --no-cpu --check 300 --e2e-reps 0 &&
$S 300 f_a12.json python -u bench.py --lib karmada_amd/libkp_a12.so --steps 200 --warmup 3 --no-cpu --check 300 --e2e-reps 0 &&
$S 400 f_b5.json python -u bench.py --config 5 --bindings 125000 --steps 20 --warmup 2 --no-cpu --check 500 --e2e-reps 2 &&
$S 300 f_b4.json python -u bench.py --config 4 --steps 50 --warmup 2 --no-cpu --check 500 --e2e-reps 2
