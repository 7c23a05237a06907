#!/bin/bash
# Tuning variant of one kernel group: kernels.hip's group TU rebuilt with extra flags,
# linked with the regular objects of every other group (never shipped as libkp.so).
#   bash tools/variant_tu.sh <name> <tu> "<-DFLAGS ...>"   -> karmada_amd/libkp_<name>.so
set -e
name=$1; tu=$2; flags=$3
cd "$(dirname "$0")/../karmada_amd/csrc"
HIPFLAGS="-std=c++17 -O3 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-lambda-capture -Wno-bitwise-instead-of-logical"
/opt/rocm/bin/hipcc $HIPFLAGS $flags -DKP_TU=$tu -c -o kernels_v${name}_tu$tu.o kernels.hip
objs=""
for t in 1 2 3 4 5 6 7 8 9 10 11 12 13; do
  if [ $t = $tu ]; then objs="$objs kernels_v${name}_tu$t.o"; else objs="$objs kernels_tu$t.o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../libkp_$name.so $objs engine.o multi.o -lpthread
echo "built karmada_amd/libkp_$name.so"
