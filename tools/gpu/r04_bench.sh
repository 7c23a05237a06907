#!/bin/bash
# Round-4 measurement batch (one gpurun call): the driver's default bench line, kernel
# statistics of config 3, the high-entropy config 10 on each route, configs 2/4/5, the
# config-5 slow-path reasons. Every step under its own time limit (tools/gpu/step.sh).
S=tools/gpu/step.sh
$S 420 b3.json python -u bench.py && \
$S 300 b10.json python -u bench.py --config 10 --steps 20 --warmup 2 --no-cpu --check 300 --e2e-reps 0 --inflight 1 && \
$S 300 b10_rows.json env KP_PAIR_ROWS=1 python -u bench.py --config 10 --steps 20 --warmup 2 --no-cpu --check 300 --e2e-reps 0 --inflight 1 && \
$S 300 b10_ord.json env KP_ORDER_AMORT=0 python -u bench.py --config 10 --steps 10 --warmup 1 --no-cpu --check 300 --e2e-reps 0 --inflight 1 && \
$S 300 b2.json python -u bench.py --config 2 --steps 20 --warmup 2 --no-cpu --check 300 --e2e-reps 2 && \
$S 300 b4.json python -u bench.py --config 4 --steps 20 --warmup 2 --no-cpu --check 300 --e2e-reps 2 && \
$S 400 b5.json python -u bench.py --config 5 --bindings 125000 --steps 10 --warmup 1 --no-cpu --check 300 --e2e-reps 2 && \
$S 200 slow5.log env KP_DEBUG_SLOW=1 DIAG_NO_ORACLE=1 python -u tools/gpu/diag_cfg8.py karmada_amd/libkp.so 5:5:10000:125000 1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof3 -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 2 --no-cpu --check 0 --e2e-reps 0 --inflight 1 > $GRAFT_REPO_ROOT/gpurun_out/prof3.log 2>&1
