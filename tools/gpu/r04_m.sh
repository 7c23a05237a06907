#!/bin/bash
# round 4: Webster quota search for few parties; GPU suite; configs 3, 5, 4, 2
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 300 m_b3.json python -u bench.py --steps 300 --warmup 5 --no-cpu --check 1000 --e2e-reps 0 &&
$S 600 m_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 400 m_b5.json python -u bench.py --config 5 --bindings 125000 --steps 20 --warmup 2 --no-cpu --check 500 --e2e-reps 0 &&
$S 300 m_b4.json python -u bench.py --config 4 --steps 50 --warmup 2 --no-cpu --check 500 --e2e-reps 0 &&
$S 300 m_b2.json python -u bench.py --config 2 --steps 50 --warmup 2 --no-cpu --check 500 --e2e-reps 0
