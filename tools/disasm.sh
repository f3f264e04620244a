#!/usr/bin/env bash
# The gfx950 disassembly of one device object (hipcc -c output):
#   tools/disasm.sh huff-encoding_amd/build/device/decode_wave.o > /tmp/dw.s
set -euo pipefail
L=/opt/rocm/lib/llvm/bin
t=$(mktemp -d)
$L/llvm-objcopy --dump-section=.hip_fatbin=$t/f.fatbin "$1" $t/h.o
tgt=$(python3 -c "import sys; sys.path.insert(0, '$(dirname "$0")'); import check_shift64 as c; print(c.TARGET)")
$L/clang-offload-bundler --unbundle --type=o --input=$t/f.fatbin --targets=$tgt --output=$t/k.co
$L/llvm-objdump -d $t/k.co
rm -rf $t
