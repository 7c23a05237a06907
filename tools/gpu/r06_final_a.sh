#!/bin/bash
# Round-6 final binary, part A: smoke, the GPU suite, the driver's exact command, the default run
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 120 fa_smoke.log python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' &&
$S 900 fa_suite.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 400 fa_driver_cmd.json python -u bench.py --gpus 1 --steps 20 --warmup 5 &&
$S 400 fa_default.json python -u bench.py
