#!/bin/bash
# Experimental library variant of ONE level count's net kernels (net_lv.hip):
# recompile it with extra defines and link it with the in-tree objects into
# _lib/libtropical_hip_<name>.so (TNP_LIB=libtropical_hip_<name>.so).
#   tools/build_lv_variant.sh <name> <levels> "-DTNP_FWD_SHADOW -DTNP_SHAPES_BENCH_ONLY"
set -e
cd "$(dirname "$0")/../tropical-nerf.pytorch_amd/csrc"
name=$1; lv=$2; defs=$3
make -s -j8 >/dev/null
objs=""
for o in build/*.o; do
  [ "$o" = "build/net_lv$lv.o" ] && continue
  objs="$objs $o"
done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-function \
  -DTNP_LV=$lv $defs -c net_lv.hip -o build/_variant_$name.o.tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../tropical/_lib/libtropical_hip_$name.so $objs \
  build/_variant_$name.o.tmp
rm -f build/_variant_$name.o.tmp
echo "built _lib/libtropical_hip_$name.so"
