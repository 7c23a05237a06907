#!/bin/bash
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 200 st_c3.log python -u tools/gpu/r06_stamps.py 3 &&
$S 200 st_c10.log python -u tools/gpu/r06_stamps.py 10
