#!/bin/bash
# pack false-sharing fix: pack scaling at 1 and 16 threads, then the bench's end-to-end legs
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
KP_PACK_THREADS=1 $S 200 d_pack_t1.log python -u tools/gpu/r06_pack.py &&
KP_PACK_THREADS=16 $S 200 d_pack_t16.log python -u tools/gpu/r06_pack.py &&
$S 300 d_bench.json python -u bench.py --no-cpu --steps 200 --e2e-reps 10
