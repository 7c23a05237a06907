#!/bin/bash
# k_select_top phase stamps at HEAD (config 3, 10); host pack scaling over thread counts,
# with and without glibc malloc's mmap/trim thresholds raised
S=tools/gpu/step.sh
rm -f gpurun_out/steps.log
$S 200 c_st3.log python -u tools/gpu/r06_stamps.py 3 &&
$S 200 c_st10.log python -u tools/gpu/r06_stamps.py 10 &&
for T in 1 4 8 16; do
  KP_PACK_THREADS=$T $S 200 c_pack_t$T.log python -u tools/gpu/r06_pack.py || exit $?
  GLIBC_TUNABLES=glibc.malloc.mmap_threshold=2000000000:glibc.malloc.trim_threshold=4000000000 KP_PACK_THREADS=$T \
    $S 200 c_pack_m_t$T.log python -u tools/gpu/r06_pack.py || exit $?
done
