#!/bin/bash
# launch arguments in device slots (no per-wave scratch copy), error results in k_select_top
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu --check 300 --e2e-reps 0"
$S 900 m_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 200 m_c4.json $B --config 4 &&
$S 300 m_c5.json $B --config 5 &&
$S 200 m_c3.json $B &&
$S 200 m_c2.json $B --config 2
