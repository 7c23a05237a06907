#!/bin/bash
# k_spread_order: region of each class-order entry beside it, entries loaded a step ahead,
# the feasibility row in LDS. GPU parity, then config 4 A/B against libkp_base.so
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 600 s_par.log python -u -m pytest tests/test_gpu_parity.py tests/test_golden_spread.py tests/test_affinities.py tests/test_h4_min_groups.py -m gpu -x -q --timeout 120 --timeout-method thread &&
for rep in 1 2 3; do
  $S 300 s_c4_new_$rep.json python -u bench.py --config 4 --steps 200 --no-cpu --check 300 --e2e-reps 0 || exit $?
  $S 300 s_c4_base_$rep.json python -u bench.py --config 4 --steps 200 --no-cpu --check 300 --e2e-reps 0 --lib karmada_amd/libkp_base.so || exit $?
done
