#!/bin/bash
# A/B builds of libnpd.so with npd_gru.hip compiled under extra flags (tools/bin/libnpd_<name>.so; loaded through
# NPD_LIB).  Usage: bash tools/build_gru_variant.sh "name:-fno-slp-vectorize" ...
set -e
cd "$(dirname "$0")/.."
make -j4 lib >/dev/null
mkdir -p tools/bin
for v in "$@"; do
  n=${v%%:*}; f=${v#*:}
  mkdir -p build/var_$n
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude \
    -Ineural_polar_decoder_amd/csrc -munsafe-fp-atomics $f \
    -c neural_polar_decoder_amd/csrc/npd_gru.hip -o build/var_$n/npd_gru.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/bin/libnpd_$n.so \
    $(ls build/obj/*.o | grep -v "/npd_gru.o") build/var_$n/npd_gru.o -Wl,--no-undefined
  echo "built tools/bin/libnpd_$n.so ($f)"
done
