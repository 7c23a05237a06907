#!/bin/bash
# round 4: relanded optimisations + iterative pdqsort: config 8 seed 6 passes, GPU suite,
# default bench, stamps of configs 5/3, kernel statistics of config 3 (CSV)
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 diag8r.log python -u tools/gpu/diag_cfg8.py karmada_amd/libkp.so 8:6:300:1500 20 &&
$S 600 gputest_r.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 420 b3r.json python -u bench.py &&
$S 300 stamps5.log python -u bench.py --lib karmada_amd/libkp_stamps.so --config 5 --bindings 125000 --steps 2 --warmup 1 --no-cpu --check 0 --inflight 1 --e2e-reps 0 &&
$S 300 stamps3.log python -u bench.py --lib karmada_amd/libkp_stamps.so --steps 2 --warmup 1 --no-cpu --check 0 --inflight 1 --e2e-reps 0 &&
cd /tmp && export TMPDIR=/tmp && mkdir -p $GRAFT_REPO_ROOT/gpurun_out/prof3r &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof3r -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 2 --no-cpu --check 0 --e2e-reps 0 --inflight 1 > $GRAFT_REPO_ROOT/gpurun_out/prof3r.log 2>&1
