#!/bin/bash
# host worker pool for the packer: pack timing at 16 threads, end-to-end legs x2
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
KP_PACK_THREADS=16 $S 200 p_pack_t16.log python -u tools/gpu/r06_pack.py &&
$S 400 p_e2e_1.json python -u bench.py --no-cpu --steps 200 --e2e-reps 10 --check 200 &&
$S 400 p_e2e_2.json python -u bench.py --no-cpu --steps 200 --e2e-reps 10 --check 200
