#!/bin/bash
# round 4: k_select_top_wg for the large-subset bindings (vs KP_TOP_WG=0); GPU suite
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 n_b3.json python -u bench.py --steps 300 --warmup 5 --no-cpu --check 1000 --e2e-reps 0 &&
$S 300 n_nowg.json env KP_TOP_WG=0 python -u bench.py --steps 300 --warmup 5 --no-cpu --check 0 --e2e-reps 0 &&
$S 400 n_b5.json python -u bench.py --config 5 --bindings 125000 --steps 20 --warmup 2 --no-cpu --check 500 --e2e-reps 0 &&
$S 600 n_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
