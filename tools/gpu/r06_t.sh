#!/bin/bash
# quota-divisor bracket in webster_par: GPU parity, stamps (bisection share), bench x2
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 600 t_par.log python -u -m pytest tests/test_gpu_blk.py tests/test_gpu_parity.py tests/test_golden_engine.py tests/test_golden_spread.py -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 200 t_st3.log python -u tools/gpu/r06_stamps.py 3 &&
$S 300 t_c3_1.json python -u bench.py --no-cpu --steps 200 --e2e-reps 0 --check 300 &&
$S 300 t_c3_2.json python -u bench.py --no-cpu --steps 200 --e2e-reps 0 --check 300
