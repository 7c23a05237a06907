#!/bin/bash
# same-box A/B: libkp_base.so (HEAD before the change) against libkp.so, config 3, alternating
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 600 j_par.log python -u -m pytest tests/test_gpu_parity.py tests/test_golden_engine.py -m gpu -x -q --timeout 120 --timeout-method thread &&
for rep in 1 2 3; do
  $S 300 j_base_$rep.json python -u bench.py --no-cpu --steps 200 --e2e-reps 0 --check 300 --lib karmada_amd/libkp_base.so || exit $?
  $S 300 j_new_$rep.json python -u bench.py --no-cpu --steps 200 --e2e-reps 0 --check 300 || exit $?
done
