#!/bin/bash
# lanes in flight: the driver's exact command at --inflight 4 / 6 / 8, interleaved, 5 runs each
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
for rep in 1 2 3 4 5; do
  for L in 4 6 8; do
    $S 300 q_l${L}_$rep.json python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-reps 0 --check 100 --inflight $L || exit $?
  done
done
