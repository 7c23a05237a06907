#!/bin/bash
# rocprofv3 kernel statistics of configs 3/4/5 and PMC passes of configs 3/4/5 (current build)
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp &&
for c in 3 4 5; do
  b=100000; [ $c = 5 ] && b=125000
  mkdir -p $R/gpurun_out/y_prof$c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/y_prof$c -o p -- python3 $R/bench.py --config $c --bindings $b --steps 30 --warmup 2 --no-cpu --check 0 --e2e-reps 0 --inflight 1 > $R/gpurun_out/y_prof$c.log 2>&1 || exit $?
done &&
cd $R && bash tools/gpu/prof_pmc.sh y3 && bash tools/gpu/prof_pmc.sh y4 --config 4 && bash tools/gpu/prof_pmc.sh y5 --config 5 --bindings 125000
