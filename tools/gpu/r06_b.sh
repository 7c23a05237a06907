#!/bin/bash
# webster_reg: device self-test, GPU parity, bench; host pack timing with kp_pack_cache
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 b_blk.log python -u -m pytest tests/test_gpu_blk.py tests/test_pack_cache.py -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 600 b_par.log python -u -m pytest tests/test_gpu_parity.py tests/test_golden_engine.py -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 300 b_driver.json python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu &&
$S 300 b_default.json python -u bench.py --no-cpu --e2e-reps 0 &&
$S 200 b_pack.log python -u tools/gpu/r06_pack.py
