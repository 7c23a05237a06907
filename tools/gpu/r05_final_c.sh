#!/bin/bash
# Round-5 final binary with 16 hardware queues: smoke, the driver's exact command, the
# default run, configs 4/5/10 (parity re-checked in every line)
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu --check 300 --e2e-reps 0"
$S 120 fc_smoke.log python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' &&
$S 400 fc_driver_cmd.json python -u bench.py --gpus 1 --steps 20 --warmup 5 &&
$S 400 fc_default.json python -u bench.py &&
$S 200 fc_c4.json $B --config 4 &&
$S 200 fc_c10.json $B --config 10 &&
$S 300 fc_c5.json $B --config 5 &&
$S 200 fc_c2.json $B --config 2
