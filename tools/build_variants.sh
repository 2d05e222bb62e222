#!/bin/bash
# A/B builds of librf.so with one translation unit compiled under extra -D flags (diagnostics; RF_LIB=<path>).
#   tools/build_variants.sh <unit.hip> name1 "flags1" name2 "flags2" ...  -> recommendflow_amd/lib/var/librf_<name>.so
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
CS="$ROOT/recommendflow_amd/csrc"; OBJ="$ROOT/recommendflow_amd/lib/obj"; VAR="$ROOT/recommendflow_amd/lib/var"
mkdir -p "$VAR"
make -s -C "$CS" >/dev/null
unit=$1; shift
base=$(basename "$unit" .hip)
others=$(ls "$OBJ"/*.o | grep -v "/$base.o$")
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -ffp-contract=off $flags \
     -c "$CS/$unit" -o "$VAR/$base.$name.o" &
done
wait
for o in "$VAR"/$base.*.o; do
  name=$(basename "$o" .o); name=${name#$base.}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$VAR/librf_$name.so" $others "$o" -lz -ldl -lpthread
  echo "built $VAR/librf_$name.so"
done
