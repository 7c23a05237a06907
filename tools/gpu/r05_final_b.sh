#!/bin/bash
# Round-5 final binary, part B: rocprofv3 kernel statistics (serial runs, each kernel's
# launches alone on the GPU) and the five PMC passes per config, default sizes
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp &&
for c in 3 4 5 10; do
  mkdir -p $R/gpurun_out/z_prof$c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/z_prof$c -o p -- python3 $R/bench.py --config $c --steps 30 --warmup 2 --no-cpu --check 0 --e2e-reps 0 --inflight 1 > $R/gpurun_out/z_prof$c.log 2>&1 || exit $?
done &&
cd $R && bash tools/gpu/prof_pmc.sh z3 && bash tools/gpu/prof_pmc.sh z4 --config 4 && bash tools/gpu/prof_pmc.sh z10 --config 10 && bash tools/gpu/prof_pmc.sh z5 --config 5
