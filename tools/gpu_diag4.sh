#!/usr/bin/env bash
# two-chain decoder: keep-address modes and u32 table (HUFF_KEEPADDR 1..4)
set -uo pipefail
out=gpurun_out/diag4; mkdir -p $out
export HUFF_ILP2=1
for m in 1 2 3 4; do
  HUFF_KEEPADDR=$m timeout -k 10 200 python tools/diag_decode.py uniform:256:10 zipf:256:10 > $out/ka$m.jsonl 2>&1 || exit 1
done
echo diag4 done
