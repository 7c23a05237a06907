#!/bin/bash
# Round-4 bisection of the config 8 seed 6 divergence: each candidate library,
# three passes over the int32-wrap universes and config 3/7 slices.
set -o pipefail
mkdir -p gpurun_out
SPECS="8:6:300:1500 8:4:64:2000 8:5:16:600 7:17:2000:3000 3:3:5000:2000"
for lib in "$@"; do
  for pass in 1 2 3; do
    echo "== $lib pass $pass" >> gpurun_out/bisect.log
    timeout -k 10 150 python -u tools/gpu/parity_lib.py "$lib" $SPECS >> gpurun_out/bisect.log 2>&1
    rc=$?
    echo "rc=$rc" >> gpurun_out/bisect.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done
