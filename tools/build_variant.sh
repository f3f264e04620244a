#!/usr/bin/env bash
# A/B library: huff-encoding_amd/lib/<name>/libhuffgpu.so = the current build
# with the listed sources (device .hip or host .cpp) recompiled with extra
# flags (CPU only; load it with HUFF_LIB_AB=<name>). Device variants must pass
# the same shift64 check.
#   tools/build_variant.sh <name> "<flags>" csrc/device/decode_wave.hip csrc/runtime/runtime.cpp [...]
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/huff-encoding_amd
name=$1; flags=$2; shift 2
W=$R/scratch/variant_$name
mkdir -p $W $P/lib/$name
repl=()
for src in "$@"; do
  case $src in
    *.hip)
      o=$W/$(basename ${src%.hip}).o
      /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -Wall -Wno-unused-result -I$R/include -I$P/csrc --offload-arch=gfx950 \
        -munsafe-fp-atomics $flags -c $P/$src -o $o
      python3 $R/tools/check_shift64.py $o
      repl+=("device/$(basename $o)");;
    *.cpp)  # host sources (runtime/, csrc/ top level) with the same flags
      o=$W/$(basename ${src%.cpp}).o
      g++ -std=c++17 -O3 -fPIC -Wall -Wno-unused-result -I$R/include -I$P/csrc -D__HIP_PLATFORM_AMD__ \
        -I/opt/rocm/include -Wno-unused-value $flags -c $P/$src -o $o
      d=$(dirname ${src#csrc/}); [ "$d" = . ] && d="" || d="$d/"
      repl+=("$d$(basename $o)");;
  esac
done
objs=""
for o in $P/build/host/*.o $P/build/runtime/*.o $P/build/*.o $P/build/device/*.o; do
  rel=${o#$P/build/}; skip=0
  for r in "${repl[@]}"; do [ "$rel" = "$r" ] && skip=1; done
  [ $skip = 0 ] && objs="$objs $o"
done
for r in "${repl[@]}"; do objs="$objs $W/$(basename $r)"; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o $P/lib/$name/libhuffgpu.so $objs \
  -Wl,-soname,libhuffgpu.so -L/opt/rocm/lib -lrccl -lpthread -Wl,-rpath,/opt/rocm/lib
echo "built lib/$name"
