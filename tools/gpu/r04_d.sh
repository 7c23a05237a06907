#!/bin/bash
# round 4: k_slow candidate order from the class orders, route-built batch lists: GPU
# suite, config 3 and 5 lines, stamps of configs 3/5, packing breakdown
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 600 d_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 300 d_b3.json python -u bench.py --steps 300 --warmup 5 --no-cpu --check 1000 --e2e-reps 3 &&
$S 400 d_b5.json python -u bench.py --config 5 --bindings 125000 --steps 20 --warmup 2 --no-cpu --check 500 --e2e-reps 2 &&
$S 300 d_b4.json python -u bench.py --config 4 --steps 50 --warmup 2 --no-cpu --check 500 --e2e-reps 2 &&
$S 300 d_stamps5.log env KP_DEBUG_SLOW=1 python -u bench.py --lib karmada_amd/libkp_stamps.so --config 5 --bindings 125000 --steps 2 --warmup 1 --no-cpu --check 0 --inflight 1 --e2e-reps 0 &&
$S 300 d_stamps3.log env KP_TOP_SPLIT=0 python -u bench.py --lib karmada_amd/libkp_stamps.so --steps 2 --warmup 1 --no-cpu --check 0 --inflight 1 --e2e-reps 0 &&
$S 200 d_pack.log python -u tools/gpu/packtime.py
