#!/usr/bin/env bash
# Builds the three libraries of the 64-bit-shift bisection (DESIGN.md §3,
# "The 64-bit shift hazard") from the round-2 wrong-letter reproducer
# (decode_wave.hip with -DHUFF_DEC_EARLY_LOADS=1), on the CPU:
#   lib/sh64A  the reproducer's assembly, reassembled unchanged
#   lib/sh64B  the same instructions, k_decode_fixed<PAD>'s allocation raised
#              from 72 to 80 VGPRs (so v72, the register after the refill
#              shift's amount v71, belongs to the wave; occupancy unchanged:
#              the LDS already caps the kernel at 6 workgroups per CU)
#   lib/sh64C  72 VGPRs, the three shifts by v71 rewritten to shift by a
#              dead register holding a copy of v71
# Every other object is the production build's.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/huff-encoding_amd
W=$R/scratch/sh64
L=/opt/rocm/lib/llvm/bin
mkdir -p $W
F=_ZN4huff3dev12_GLOBAL__N_114k_decode_fixedILb1EEEvNS0_10DecodeArgsE
FL="-std=c++17 -O3 -I$R/include -I$P/csrc --offload-arch=gfx950 -munsafe-fp-atomics -fPIC -DHUFF_DEC_EARLY_LOADS=1"
/opt/rocm/bin/hipcc $FL --cuda-device-only -S -o $W/repro.s $P/csrc/device/decode_wave.hip 2>/dev/null
/opt/rocm/bin/hipcc $FL -c -o $W/host.o $P/csrc/device/decode_wave.hip 2>/dev/null
python3 - "$W" "$F" <<'PY'
import re, sys
w, f = sys.argv[1], sys.argv[2]
src = open(f"{w}/repro.s").read().split("\n")
# kernel body range, its descriptor and its metadata
start = src.index(f"{f}: ; @{f}")
end = next(i for i in range(start, len(src)) if src[i].startswith(".Lfunc_end"))
open(f"{w}/A.s", "w").write("\n".join(src))
# B: allocation 72 -> 80 (descriptor + metadata), instructions untouched
b = list(src)
kd = b.index(f"\t.amdhsa_kernel {f}")
for i in range(kd, kd + 60):
    b[i] = b[i].replace(".amdhsa_next_free_vgpr 72", ".amdhsa_next_free_vgpr 80").replace(".amdhsa_accum_offset 72", ".amdhsa_accum_offset 80")
    if b[i].startswith("\t.end_amdhsa_kernel"):
        break
b = [l.replace(f"{f}.num_vgpr, 72", f"{f}.num_vgpr, 80") for l in b]
md = next(i for i in range(len(b)) if b[i].strip() == f".name:           {f}")
for i in range(md - 40, md + 40):
    if b[i].strip() == ".vgpr_count:     72":
        b[i] = b[i].replace("72", "80")
open(f"{w}/B.s", "w").write("\n".join(b))
# C: shift amounts moved off v71 (the copy goes to a register the next
# instructions overwrite anyway)
c = list(src)
n = 0
for i in range(start, end):
    m = re.match(r"^\tv_lshrrev_b64 v\[(\d+):(\d+)\], v71, (v\[\d+:\d+\])$", c[i])
    if not m:
        continue
    lo, hi, s = int(m.group(1)), int(m.group(2)), m.group(3)
    if s != f"v[{lo}:{hi}]":
        tmp = lo            # the destination's low half: dead until written
    else:
        # the source is the destination: the next VALU write of another register
        nxt = c[i + 2].split()
        assert nxt[0] == "v_lshrrev_b32_e32", c[i + 2]
        tmp = int(nxt[1].rstrip(",")[1:])
    c[i] = f"\tv_mov_b32_e32 v{tmp}, v71\n\tv_lshrrev_b64 v[{lo}:{hi}], v{tmp}, {s}"
    n += 1
assert n == 3, n
open(f"{w}/C.s", "w").write("\n".join(c))
PY
for v in A B C; do
  $L/clang -x assembler -target amdgcn-amd-amdhsa -mcpu=gfx950 -c $W/$v.s -o $W/$v.dev.o
  $L/ld.lld -shared $W/$v.dev.o -o $W/$v.co
  $L/clang-offload-bundler --type=o --targets=host-x86_64-unknown-linux-gnu-,hipv4-amdgcn-amd-amdhsa--gfx950 \
    --input=/dev/null --input=$W/$v.co --output=$W/$v.fatbin
  cp $W/host.o $W/$v.o
  $L/llvm-objcopy --update-section .hip_fatbin=$W/$v.fatbin $W/$v.o
  objs=$(ls $P/build/host/*.o $P/build/runtime/*.o $P/build/*.o $P/build/device/*.o | grep -v device/decode_wave.o)
  mkdir -p $P/lib/sh64$v
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o $P/lib/sh64$v/libhuffgpu.so $objs $W/$v.o \
    -Wl,-soname,libhuffgpu.so -L/opt/rocm/lib -lrccl -lpthread -Wl,-rpath,/opt/rocm/lib
  echo "built lib/sh64$v"
done
python3 $R/tools/check_shift64.py $W/A.co $W/B.co $W/C.co || true
