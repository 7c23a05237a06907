#!/bin/bash
# round 4: k_slow launched after the flagged count is read back (none: no launch), request
# memo in the packer: GPU suite, configs 3 (default command) / 4 / 5, packing breakdown
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 600 o_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 420 o_default.json python -u bench.py &&
$S 300 o_b4.json python -u bench.py --config 4 --steps 50 --warmup 2 --no-cpu --check 300 --e2e-reps 2 &&
$S 400 o_b5.json python -u bench.py --config 5 --bindings 125000 --steps 20 --warmup 2 --no-cpu --check 300 --e2e-reps 2 &&
$S 200 o_pack.log python -u tools/gpu/packtime.py &&
$S 300 o_diag8.log python -u tools/gpu/diag_cfg8.py karmada_amd/libkp.so 8:6:300:1500 10
