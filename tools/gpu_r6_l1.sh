#!/usr/bin/env bash
# Round 6: k_decode_fixed's short-code region (DecodeArgs::l1_mask) against
# the plain table (HUFF_DEC_L1=0), alternated on one box: the indexed decode
# and the index-free pipeline on 1 GiB Zipf and text, the general kernels on
# uniform (no short codes: region off either way).
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r6l1}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
for r in 1 2; do
  for wl in zipf text; do
    for l1 in 1 0; do
      HUFF_DEC_L1=$l1 timeout -k 10 120 python -u tools/kbench.py --phase decode --workload $wl --iters 20 > $out/dec_${wl}_l1${l1}_$r.json 2> $out/dec_${wl}_l1${l1}_$r.err || { tail -5 $out/dec_${wl}_l1${l1}_$r.err; exit 1; }
      HUFF_DEC_L1=$l1 timeout -k 10 120 python -u tools/kbench.py --phase indexless --workload $wl --iters 10 > $out/idx_${wl}_l1${l1}_$r.json 2> $out/idx_${wl}_l1${l1}_$r.err || { tail -5 $out/idx_${wl}_l1${l1}_$r.err; exit 1; }
    done
  done
done
grep -H . $out/*.json | sed "s|$out/||"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof_zipf -o run --output-format csv -- python3 $root/tools/kbench.py --phase decode --workload zipf --iters 10 > $out/prof_zipf.log 2>&1 || { tail -5 $out/prof_zipf.log; exit 1; }
grep -h "k_decode" $out/prof_zipf/run_kernel_stats.csv | cut -c1-150
