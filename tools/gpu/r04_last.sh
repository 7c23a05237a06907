#!/bin/bash
# round 4, exact final binary: GPU suite, smoke(), default bench line
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 600 last_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S 300 last_smoke.log python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" &&
$S 420 last_default.json python -u bench.py
