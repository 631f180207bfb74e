#!/bin/bash
# A/B builds of libkgat_hip.so: tools/build_variants.sh SRC.hip NAME1:"-DFLAG=1" NAME2:"-DFLAG=2" ...
# -> variants/libkgat_NAME.so (every other object from the regular build).  Select one at run
# time with KGAT_HIP_LIB=variants/libkgat_NAME.so.
set -eu
cd "$(dirname "$0")/.."
C=problem-recommender-system-using-kgat-in-codeforces_amd/csrc
make -C $C -j8 > /dev/null
src=$1; shift
base=$(basename $src .hip)
mkdir -p variants
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -I include -I $C $flags -c $C/$src -o /tmp/v_$name.o
  objs=$(ls $C/build/*.o | grep -v "/$base.o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o variants/libkgat_$name.so $objs /tmp/v_$name.o -pthread
  echo "variants/libkgat_$name.so"
done
