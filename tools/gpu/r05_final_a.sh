#!/bin/bash
# Round-5 final binary, part A: GPU suite, smoke, the driver's exact bench command, the
# default 500-step run, and the other configs' lines (parity re-checked in every line)
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu --check 300 --e2e-reps 0"
$S 900 fa_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 120 fa_smoke.log python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' &&
$S 400 fa_driver_cmd.json python -u bench.py --gpus 1 --steps 20 --warmup 5 &&
$S 400 fa_default.json python -u bench.py &&
$S 200 fa_c1.json $B --config 1 &&
$S 200 fa_c2.json $B --config 2 &&
$S 200 fa_c4.json $B --config 4 &&
$S 300 fa_c5.json $B --config 5 &&
$S 200 fa_c10.json $B --config 10
