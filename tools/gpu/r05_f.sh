#!/bin/bash
# k_select_top split: phase stamps, per-dispatch kernel trace (small / large slice), KP_TOP_WG line
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
export TMPDIR=/tmp
$S 300 f_st3.log python -u bench.py --lib karmada_amd/libkp_stamps.so --config 3 --steps 2 --warmup 1 --no-cpu --check 0 --inflight 1 --e2e-reps 0 &&
$S 300 f_kt.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/f_kt -o kt -- python bench.py --steps 3 --warmup 1 --no-cpu --check 0 --inflight 1 --e2e-reps 0 &&
$S 200 f_wg.json env KP_TOP_WG=1 python -u bench.py --steps 100 --warmup 5 --no-cpu --check 300 --e2e-reps 0
