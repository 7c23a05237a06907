#!/bin/bash
# round 4: the iterative pdqsort_go build on config 8 seed 6 (repeated passes), then the GPU suite
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 diag8.log python -u tools/gpu/diag_cfg8.py karmada_amd/libkp.so 8:6:300:1500 30 &&
$S 240 diag8b.log python -u tools/gpu/diag_cfg8.py karmada_amd/libkp.so 8:6:1000:4000 8 &&
$S 600 gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
