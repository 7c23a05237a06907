#!/bin/bash
# round 4: k_select_top launch placement (two streams vs one), occupancy variant, packing
# breakdown, the RCCL path at world size 1, config-3 kernel statistics
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 c_split.json python -u bench.py --steps 200 --warmup 5 --no-cpu --check 1000 --e2e-reps 3 &&
$S 300 c_nosplit.json env KP_TOP_SPLIT=0 python -u bench.py --steps 200 --warmup 5 --no-cpu --check 0 --e2e-reps 0 &&
$S 300 c_mw5.json python -u bench.py --lib karmada_amd/libkp_mw5.so --steps 200 --warmup 5 --no-cpu --check 1000 --e2e-reps 0 &&
$S 300 c_mw5_nosplit.json env KP_TOP_SPLIT=0 python -u bench.py --lib karmada_amd/libkp_mw5.so --steps 200 --warmup 5 --no-cpu --check 0 --e2e-reps 0 &&
$S 200 c_pack.log python -u tools/gpu/packtime.py &&
$S 300 c_rccl.json env KP_DIST_FORCE=1 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --steps 50 --warmup 2 --no-cpu --check 300 --e2e-reps 0 &&
cd /tmp && export TMPDIR=/tmp && mkdir -p $GRAFT_REPO_ROOT/gpurun_out/prof3c &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof3c -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 2 --no-cpu --check 0 --e2e-reps 0 --inflight 1 > $GRAFT_REPO_ROOT/gpurun_out/prof3c.log 2>&1
