#!/bin/bash
# Round 6: GPU suite, the driver's exact bench command, the default bench
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 900 a_tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 300 a_driver.json python -u bench.py --gpus 1 --steps 20 --warmup 5 &&
$S 300 a_default.json python -u bench.py --no-cpu
