#!/bin/bash
# webster_reg inside webster_par for compacted lists of <= 64 (k_select_top's large subsets)
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 600 i_par.log python -u -m pytest tests/test_gpu_blk.py tests/test_gpu_parity.py tests/test_golden_engine.py -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 300 i_c3a.json python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu &&
$S 300 i_c3b.json python -u bench.py --no-cpu --steps 200 --e2e-reps 0 &&
$S 200 i_st3.log python -u tools/gpu/r06_stamps.py 3
