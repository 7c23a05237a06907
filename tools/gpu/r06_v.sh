#!/bin/bash
# waves per workgroup of k_select_static / k_spread_order / k_region_a_order: 4 (libkp.so),
# 2 (libkp_s2.so), 1 (libkp_s1.so), same box; GPU parity of the k_select_top one-wave build
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 600 v_par.log python -u -m pytest tests/test_gpu_parity.py tests/test_golden_engine.py tests/test_gpu_blk.py -m gpu -x -q --timeout 120 --timeout-method thread &&
for c in 2 4; do
  for L in "" s2 s1; do
    lib=""; [ -n "$L" ] && lib="--lib karmada_amd/libkp_$L.so"
    $S 300 v_c${c}_${L:-s4}.json python -u bench.py --config $c --no-cpu --steps 100 --e2e-reps 0 --check 300 $lib || exit $?
  done
done
for L in "" s1; do
  lib=""; [ -n "$L" ] && lib="--lib karmada_amd/libkp_$L.so"
  $S 400 v_c5_${L:-s4}.json python -u bench.py --config 5 --no-cpu --steps 20 --e2e-reps 0 --check 300 $lib || exit $?
done
