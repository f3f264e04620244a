#!/usr/bin/env bash
# two-chain decoder failure experiments (see DESIGN.md §3 "co-resident wrong letters")
set -uo pipefail
out=gpurun_out/diag3; mkdir -p $out
export HUFF_ILP2=1
timeout -k 10 200 python tools/diag_decode.py uniform:256:10 > $out/base.jsonl 2>&1 || exit 1
HUFF_KEEPADDR=1 timeout -k 10 200 python tools/diag_decode.py uniform:256:10 > $out/keepaddr.jsonl 2>&1 || exit 1
HUFF_LIB_AB=fz timeout -k 10 300 python tools/diag_decode.py uniform:256:10 > $out/forcezero.jsonl 2>&1 || exit 1
echo diag3 done
