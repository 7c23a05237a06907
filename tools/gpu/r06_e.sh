#!/bin/bash
# fallback launches gated on read-back counts (KP_GATE_FB): GPU parity, configs 3/4/5 A/B
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 600 e_par.log python -u -m pytest tests/test_gpu_parity.py tests/test_golden_engine.py tests/test_affinities.py -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 300 e_c3.json python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu &&
for G in 1 0; do
  KP_GATE_FB=$G $S 300 e_c4_g$G.json python -u bench.py --config 4 --steps 200 --no-cpu --check 300 --e2e-reps 0 || exit $?
  KP_GATE_FB=$G $S 400 e_c5_g$G.json python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu --check 300 --e2e-reps 0 || exit $?
done
bash tools/gpu/prof_pmc.sh r06c4 --config 4
