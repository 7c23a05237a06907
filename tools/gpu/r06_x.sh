#!/bin/bash
# GPU suite on the rebuilt binary, then the driver's command with polling vs blocking host waits
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 600 fx_suite.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
for r in 1 2 3 4; do
  $S 200 x_poll_$r.json python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-reps 0 || exit 1
  KP_SYNC_BLOCK=1 $S 200 x_block_$r.json python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-reps 0 || exit 1
done
