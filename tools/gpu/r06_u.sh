#!/bin/bash
# k_select_top waves per workgroup: 2 (libkp.so) vs 1 (libkp_w1.so) vs 4 (libkp_w4.so), same box,
# default 200-step runs interleaved (serial k_select_top time and the pipelined line)
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
for rep in 1 2; do
  $S 300 u_w2_$rep.json python -u bench.py --no-cpu --steps 200 --e2e-reps 0 --check 300 || exit $?
  $S 300 u_w1_$rep.json python -u bench.py --no-cpu --steps 200 --e2e-reps 0 --check 300 --lib karmada_amd/libkp_w1.so || exit $?
  $S 300 u_w4_$rep.json python -u bench.py --no-cpu --steps 200 --e2e-reps 0 --check 300 --lib karmada_amd/libkp_w4.so || exit $?
done
