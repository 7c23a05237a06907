#!/bin/bash
# GPU suite + the world-1 RCCL bench leg on its own (verbose logs under gpurun_out/)
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 900 r5_gputest.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread &&
$S 120 r5_smoke.log python -c 'import __graft_entry__ as g; g.smoke()'
