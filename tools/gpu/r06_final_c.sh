#!/bin/bash
# Round-6 binary, part C: the other BASELINE configs (parity re-checked in every line)
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu --check 300 --e2e-reps 0"
$S 200 fc_c2.json $B --config 2 &&
$S 200 fc_c4.json $B --config 4 &&
$S 200 fc_c10.json $B --config 10 &&
$S 300 fc_c5.json $B --config 5 --steps 20 &&
$S 200 fc_c1.json $B --config 1 --steps 500
