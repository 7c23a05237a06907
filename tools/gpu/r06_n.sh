#!/bin/bash
# two batches per lane (kp_schedule_batch_submit / _collect) against one, the driver's exact
# command alternating, plus the submit/collect GPU tests
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 n_tests.log python -u -m pytest tests/test_submit_collect.py -m gpu -x -q --timeout 120 --timeout-method thread &&
for rep in 1 2 3 4; do
  $S 300 n_pl2_$rep.json python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-reps 0 --check 200 || exit $?
  $S 300 n_pl1_$rep.json python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-reps 0 --check 200 --per-lane 1 || exit $?
done
$S 300 n_pl2_long.json python -u bench.py --no-cpu --e2e-reps 0 --check 200
