#!/bin/bash
# Round 6: streams per engine x batches in flight under HIP's default 4 hardware queues
# (the GPU boxes' setting), against the round-5 layout (3 streams x 4 lanes) at 4 and 16
# queues; every line on the same box, interleaved twice.
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 200 --warmup 5 --no-cpu --check 300 --e2e-reps 0"
for rep in 1 2; do
  GPU_MAX_HW_QUEUES=4 KP_STREAMS=3 $S 200 s_q4_s3_l4_$rep.json $B --inflight 4 &&
  GPU_MAX_HW_QUEUES=4 KP_STREAMS=1 $S 200 s_q4_s1_l4_$rep.json $B --inflight 4 &&
  GPU_MAX_HW_QUEUES=4 KP_STREAMS=2 $S 200 s_q4_s2_l2_$rep.json $B --inflight 2 &&
  GPU_MAX_HW_QUEUES=4 KP_STREAMS=2 $S 200 s_q4_s2_l4_$rep.json $B --inflight 4 &&
  GPU_MAX_HW_QUEUES=4 KP_STREAMS=1 $S 200 s_q4_s1_l3_$rep.json $B --inflight 3 &&
  GPU_MAX_HW_QUEUES=4 KP_STREAMS=1 $S 200 s_q4_s1_l6_$rep.json $B --inflight 6 &&
  GPU_MAX_HW_QUEUES=16 KP_STREAMS=3 $S 200 s_q16_s3_l4_$rep.json $B --inflight 4 || exit $?
done
