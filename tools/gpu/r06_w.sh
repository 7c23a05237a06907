#!/bin/bash
# k_select_top's Webster party list capacity (KP_TOP_ECAP 160 / 320 / 480), interleaved, config 3 and 10
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
B="python -u bench.py --no-cpu --steps 100 --warmup 5 --e2e-reps 0"
for r in 1 2; do
  for v in base e320 e480; do
    L=karmada_amd/libkp.so; [ $v != base ] && L=karmada_amd/libkp_$v.so
    $S 200 w_${v}_c3_$r.json $B --lib $L --check 1000 || exit 1
  done
done
for v in base e320 e480; do
  L=karmada_amd/libkp.so; [ $v != base ] && L=karmada_amd/libkp_$v.so
  $S 200 w_${v}_c10.json $B --lib $L --config 10 --check 300 || exit 1
  $S 200 w_${v}_c5.json $B --lib $L --config 5 --steps 10 --check 300 || exit 1
done
