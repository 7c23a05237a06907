#!/bin/bash
# round 4 final build: GPU suite, default bench line, config 8 seed 6 passes, kernel
# statistics and PMC passes of config 3
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
R=$GRAFT_REPO_ROOT
$S 600 z2_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 420 z2_default.json python -u bench.py &&
$S 300 z2_diag8.log python -u tools/gpu/diag_cfg8.py karmada_amd/libkp.so 8:6:300:1500 10 &&
cd /tmp && export TMPDIR=/tmp && mkdir -p $R/gpurun_out/z2_prof3 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/z2_prof3 -o p -- python3 $R/bench.py --steps 30 --warmup 2 --no-cpu --check 0 --e2e-reps 0 --inflight 1 > $R/gpurun_out/z2_prof3.log 2>&1 &&
cd $R && bash tools/gpu/prof_pmc.sh z2
