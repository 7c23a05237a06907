#!/bin/bash
# singleton classes, one wave per class (k_est_feas_*): config 10 parity and lines, A/B
# against the workgroup form (KP_EST_FEAS_WG=1)
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 r_par.log python -u -m pytest tests/test_gpu_parity.py tests/test_submit_collect.py -m gpu -x -q --timeout 120 --timeout-method thread &&
for rep in 1 2; do
  $S 300 r_c10_w_$rep.json python -u bench.py --config 10 --steps 100 --no-cpu --check 300 --e2e-reps 0 || exit $?
  KP_EST_FEAS_WG=1 $S 300 r_c10_g_$rep.json python -u bench.py --config 10 --steps 100 --no-cpu --check 300 --e2e-reps 0 || exit $?
done
