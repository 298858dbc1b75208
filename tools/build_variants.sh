#!/bin/bash
# A/B builds of libnpd.so with ONE source file compiled under experiment macros (tools/bin/libnpd_<name>.so, loaded
# through NPD_LIB).  Usage: bash tools/build_variants.sh npd_gru "name:-DNPD_GRU16_ORDER=1" ...
set -e
cd "$(dirname "$0")/.."
src=$1; shift
make -j8 lib >/dev/null
mkdir -p tools/bin
extra=""
case $src in npd_sc*|npd_scl) extra=-fno-honor-nans;; esac
for v in "$@"; do
  n=${v%%:*}; f=${v#*:}
  mkdir -p build/var_$n
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude \
    -Ineural_polar_decoder_amd/csrc -munsafe-fp-atomics $extra $f \
    -c neural_polar_decoder_amd/csrc/$src.hip -o build/var_$n/$src.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/bin/libnpd_$n.so \
    $(ls build/obj/*.o | grep -v "/$src.o") build/var_$n/$src.o -Wl,--no-undefined
  echo "built tools/bin/libnpd_$n.so ($f)"
done
