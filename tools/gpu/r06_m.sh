#!/bin/bash
# speculative CSR copy (KP_SPEC_COPY): parity, then the driver's
# exact command alternating it on / off (m_zc1 = on), gaps recorded
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 600 m_par.log python -u -m pytest tests/test_gpu_parity.py tests/test_golden_engine.py tests/test_affinities.py -m gpu -x -q --timeout 120 --timeout-method thread &&
for rep in 1 2 3 4; do
  $S 300 m_zc1_$rep.json python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-reps 0 --check 200 || exit $?
  KP_SPEC_COPY=0 $S 300 m_zc0_$rep.json python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-reps 0 --check 200 || exit $?
done
