#!/bin/bash
# bench.py with blocking host waits by default: smoke, the driver's exact command three times
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 120 fy_smoke.log python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' &&
$S 400 fy_driver_cmd_1.json python -u bench.py --gpus 1 --steps 20 --warmup 5 &&
$S 300 fy_driver_cmd_2.json python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu &&
$S 300 fy_driver_cmd_3.json python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
