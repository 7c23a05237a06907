#!/bin/bash
# singleton classes with the feasible clusters compacted in LDS: config 10 A/B; stamps config 3
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 h_par.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "10 or config" &&
for rep in 1 2; do
  for E in 1 0; do
    KP_EST_SINGLE=$E $S 300 h_c10_e${E}_$rep.json python -u bench.py --config 10 --steps 100 --no-cpu --check 300 --e2e-reps 0 || exit $?
  done
done
$S 200 h_st3.log python -u tools/gpu/r06_stamps.py 3
