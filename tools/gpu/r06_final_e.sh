#!/bin/bash
# Final binary (one wave per k_select_top workgroup): smoke, GPU suite, the driver's exact command
# twice, the default run, kernel statistics (one stream) and PMC passes for config 3
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
R=$GRAFT_REPO_ROOT
$S 120 fe_smoke.log python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' &&
$S 900 fe_suite.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 400 fe_driver_cmd.json python -u bench.py --gpus 1 --steps 20 --warmup 5 &&
$S 300 fe_driver_cmd2.json python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu &&
$S 400 fe_default.json python -u bench.py --no-cpu
