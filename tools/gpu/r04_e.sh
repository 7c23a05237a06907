#!/bin/bash
# round 4: packing fixes + k_slow order estimates: GPU suite, config 3/5 lines, k_select_top
# phase cut-off variants (timing only), packing breakdown
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 600 e_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 300 e_b3.json python -u bench.py --steps 300 --warmup 5 --no-cpu --check 1000 --e2e-reps 3 &&
$S 200 e_pack.log python -u tools/gpu/packtime.py &&
$S 300 e_x1.json python -u bench.py --lib karmada_amd/libkp_e1.so --steps 100 --warmup 3 --no-cpu --check 0 --e2e-reps 0 &&
$S 300 e_x2.json python -u bench.py --lib karmada_amd/libkp_e2.so --steps 100 --warmup 3 --no-cpu --check 0 --e2e-reps 0 &&
$S 400 e_b5.json python -u bench.py --config 5 --bindings 125000 --steps 20 --warmup 2 --no-cpu --check 500 --e2e-reps 2 &&
$S 300 e_stamps5.log env KP_DEBUG_SLOW=1 python -u bench.py --lib karmada_amd/libkp_stamps.so --config 5 --bindings 125000 --steps 2 --warmup 1 --no-cpu --check 0 --inflight 1 --e2e-reps 0
