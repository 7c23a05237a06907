#!/bin/bash
# run-to-run spread of the driver's exact command with the completion gaps recorded
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
for rep in 1 2 3 4; do
  $S 300 l_s03_$rep.json python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-reps 0 --check 100 || exit $?
  KP_BENCH_SETTLE_S=1.0 $S 300 l_s10_$rep.json python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-reps 0 --check 100 || exit $?
done
