#!/bin/bash
# enumeration without per-party divisions: GPU parity + device self-test; end-to-end legs x2
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 600 o_par.log python -u -m pytest tests/test_gpu_blk.py tests/test_gpu_parity.py tests/test_golden_engine.py -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 400 o_e2e_1.json python -u bench.py --no-cpu --steps 200 --e2e-reps 10 --check 200 &&
$S 400 o_e2e_2.json python -u bench.py --no-cpu --steps 200 --e2e-reps 10 --check 200
