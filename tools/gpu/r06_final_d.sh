#!/bin/bash
# Final binary: rocprofv3 kernel statistics for config 3 (one stream) and its five PMC passes
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/x_prof3
cd /tmp && export TMPDIR=/tmp &&
KP_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/x_prof3 -o p -- python3 $R/bench.py --config 3 --steps 30 --warmup 2 --no-cpu --check 0 --e2e-reps 0 --inflight 1 > $R/gpurun_out/x_prof3.log 2>&1 &&
cd $R && bash tools/gpu/prof_pmc.sh x3
