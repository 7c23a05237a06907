#!/bin/bash
# GPU suite + smoke + the config 3/4/5/10 bench lines with parity samples
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu --check 300 --e2e-reps 0"
$S 900 r5e_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 120 r5e_smoke.log python -c 'import __graft_entry__ as g; g.smoke()' &&
$S 200 e_c3.json $B &&
$S 200 e_c4.json $B --config 4 &&
$S 200 e_c5.json $B --config 5 &&
$S 200 e_c10.json $B --config 10
