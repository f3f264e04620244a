#!/usr/bin/env bash
# Round 6: the persistent LDS-DMA decoder (k_decode_dma) against the one-shot
# register-staged one (HUFF_DMA_DECODE=0): the decode tests first, then
# alternated same-box kbench runs of the indexed and the index-free decode
# (each verifies its output); uniform through the general kernels too.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-dma}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 400 python -u -m pytest tests/test_gpu_indexfree.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for wl in zipf text; do
  for ph in decode indexless; do
    for r in 1 2; do
      for c in 0 1; do
        HUFF_DMA_DECODE=$c timeout -k 10 120 python tools/kbench.py --phase $ph --workload $wl --iters 10 > $out/${ph}_${wl}_d${c}_$r.json 2>> $out/err.log || { tail -5 $out/err.log; exit 1; }
        echo "$ph $wl dma=$c: $(cat $out/${ph}_${wl}_d${c}_$r.json)"
      done
    done
  done
done
for r in 1 2; do
  for c in 0 1; do
    HUFF_DISABLE_FIXED8=1 HUFF_DMA_DECODE=$c timeout -k 10 120 python tools/kbench.py --phase decode --workload uniform --iters 10 > $out/decode_uniformg_d${c}_$r.json 2>> $out/err.log || { tail -5 $out/err.log; exit 1; }
    echo "decode uniform(general) dma=$c: $(cat $out/decode_uniformg_d${c}_$r.json)"
  done
done
