#!/bin/bash
# run-to-run spread of the driver's exact command (5 runs), with and without the settle pause
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
for rep in 1 2 3; do
  $S 300 k_settle_$rep.json python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-reps 0 || exit $?
  KP_BENCH_SETTLE_S=0 $S 300 k_nosettle_$rep.json python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-reps 0 || exit $?
done
