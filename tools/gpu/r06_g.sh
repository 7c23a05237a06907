#!/bin/bash
# singleton estimator classes (feasible-only rows) at config 10: parity, A/B; k_select_top stamps
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 600 g_par.log python -u -m pytest tests/test_gpu_parity.py tests/test_golden_engine.py -m gpu -x -q --timeout 120 --timeout-method thread &&
for rep in 1 2; do
  for E in 1 0; do
    KP_EST_SINGLE=$E $S 300 g_c10_e${E}_$rep.json python -u bench.py --config 10 --steps 100 --no-cpu --check 300 --e2e-reps 0 || exit $?
  done
done
$S 200 g_st3.log python -u tools/gpu/r06_stamps.py 3
