#!/bin/bash
# histogram path of k_select_top: its GPU parity tests, config 10 and config 3 lines
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 600 r5c_tests.log python -u -m pytest tests/test_gpu_parity.py tests/test_golden_spread.py tests/test_h4_min_groups.py -m gpu -x -v --timeout 120 --timeout-method thread -k "histogram or spread or h4 or config" &&
$S 300 r5c_c10.json python -u bench.py --config 10 --steps 40 --warmup 3 --no-cpu --check 500 --e2e-reps 0 &&
$S 300 r5c_c3.json python -u bench.py --steps 200 --warmup 5 --no-cpu --check 500 --e2e-reps 0
