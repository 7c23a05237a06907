#!/bin/bash
# Round-6 binary, part B: rocprofv3 kernel statistics for configs 3/4/10, every launch on one
# stream (KP_STREAMS=1: each launch alone on the GPU, as the line times it); PMC: prof_pmc.sh
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp &&
for c in 3 4 10; do
  mkdir -p $R/gpurun_out/y_prof$c
  KP_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/y_prof$c -o p -- python3 $R/bench.py --config $c --steps 30 --warmup 2 --no-cpu --check 0 --e2e-reps 0 --inflight 1 > $R/gpurun_out/y_prof$c.log 2>&1 || exit $?
done &&
true
