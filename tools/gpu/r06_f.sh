#!/bin/bash
# KP_GATE_FB A/B: 1 (all fallbacks gated), 2 (SEL_ALL / cluster only), 0 (none), configs 4 and 5
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
for rep in 1 2; do
  for G in 1 2 0; do
    KP_GATE_FB=$G $S 300 f_c4_g${G}_$rep.json python -u bench.py --config 4 --steps 200 --no-cpu --check 100 --e2e-reps 0 || exit $?
  done
  for G in 1 2; do
    KP_GATE_FB=$G $S 400 f_c5_g${G}_$rep.json python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu --check 100 --e2e-reps 0 || exit $?
  done
done
