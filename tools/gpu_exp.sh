#!/usr/bin/env bash
# Wrong-letter reproducer ("Co-resident wrong letters"): the
# device-job cases that fail under the HUFF_DEC_EARLY_LOADS build, run against
# several builds of the same source. Build the libraries first (in the
# container), e.g.:
#   make -C huff-encoding_amd BUILD=/tmp/b_repro LIB=$PWD/huff-encoding_amd/lib/repro/libhuffgpu.so \
#        DEVEXTRA=-DHUFF_DEC_EARLY_LOADS=1
#   ... DEVEXTRA="-DHUFF_DEC_EARLY_LOADS=1 -Xarch_device -mllvm=-amdgpu-snop-padding=4"  (lib/nop)
#   ... DEVEXTRA="-DHUFF_DEC_EARLY_LOADS=1 -Xarch_device -mllvm=-amdgpu-waitcnt-forcezero" (lib/fz)
# then: tools/gpu_exp.sh repro nop fz   (each name = a lib/<name> directory)
set -uo pipefail
out=gpurun_out/exp; mkdir -p $out
sel="test_device_job_medium and (uniform or zipf) and (auto or fixed)"
for name in production "$@"; do
  if [ $name = production ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$name; fi
  timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "$sel" > $out/$name.log 2>&1
  rc=$?; echo "$name rc=$rc: $(tail -1 $out/$name.log)"
  [ $rc -le 1 ] || exit 1
done
echo "exp done"
