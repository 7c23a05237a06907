#!/bin/bash
# round 4 measurement batch: GPU suite, the driver's default bench line, configs 2/4/5,
# rocprofv3 kernel statistics of configs 3/4/5 (CSV), PMC passes of config 3
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
R=$GRAFT_REPO_ROOT
$S 600 z_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 420 z_default.json python -u bench.py &&
$S 300 z_b2.json python -u bench.py --config 2 --steps 50 --warmup 2 --check 300 --e2e-reps 2 &&
$S 300 z_b4.json python -u bench.py --config 4 --steps 50 --warmup 2 --check 300 --e2e-reps 2 &&
$S 400 z_b5.json python -u bench.py --config 5 --bindings 125000 --steps 20 --warmup 2 --check 300 --e2e-reps 2 &&
cd /tmp && export TMPDIR=/tmp &&
for c in 3 4 5; do
  b=100000; [ $c = 5 ] && b=125000
  mkdir -p $R/gpurun_out/z_prof$c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/z_prof$c -o p -- python3 $R/bench.py --config $c --bindings $b --steps 30 --warmup 2 --no-cpu --check 0 --e2e-reps 0 --inflight 1 > $R/gpurun_out/z_prof$c.log 2>&1 || exit $?
done &&
cd $R && bash tools/gpu/prof_pmc.sh z3
