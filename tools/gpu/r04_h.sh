#!/bin/bash
# round 4: k_select_top without the other strategies' code (sel_all_fast<kDynOnly>)
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 h_b3.json python -u bench.py --steps 300 --warmup 5 --no-cpu --check 1000 --e2e-reps 0 &&
$S 400 h_b5.json python -u bench.py --config 5 --bindings 125000 --steps 20 --warmup 2 --no-cpu --check 500 --e2e-reps 0 &&
$S 600 h_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
