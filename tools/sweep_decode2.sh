#!/usr/bin/env bash
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/calib > gpurun_out/calib.log 2>&1
for w in zipf text; do for cfg in "0 12" "0 11" "0 10" "2 12" "2 10" "1 12"; do
  set -- $cfg
  r=$(HUFF_DISABLE_FIXED8=1 HUFF_DEC_VARIANT=$1 HUFF_DEC_MS_BITS=$2 timeout -k 10 120 python tools/kbench.py --phase decode --workload $w --iters 20)
  echo "w=$w v=$1 K=$2 $r"
done; done > gpurun_out/dec_sweep2.log 2>&1
HUFF_DEC_VARIANT=0 bash tools/profile.sh decode zipf ms_dec_zipf > /dev/null
python tools/summarize_prof.py gpurun_out/prof/ms_dec_zipf > gpurun_out/ms_dec_zipf.json
