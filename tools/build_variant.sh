#!/bin/bash
# Experimental library variant: recompile ONE source with extra defines and
# link it with the in-tree objects into _lib/libtropical_hip_<name>.so
# (selected at run time by TNP_LIB=libtropical_hip_<name>.so).
#   tools/build_variant.sh <name> <source.hip> "-DFOO -DBAR"
set -e
cd "$(dirname "$0")/../tropical-nerf.pytorch_amd/csrc"
name=$1; src=$2; defs=$3
make -s -j8 >/dev/null
objs=""
for o in build/*.o; do
  [ "$o" = "build/$src.o" ] && continue
  objs="$objs $o"
done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-function $defs \
  -c $src -o build/_variant_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../tropical/_lib/libtropical_hip_$name.so $objs build/_variant_$name.o
rm -f build/_variant_$name.o
echo "built _lib/libtropical_hip_$name.so"
