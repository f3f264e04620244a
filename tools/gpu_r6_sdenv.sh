#!/usr/bin/env bash
# Round 6: the one-pass index-free decoder under environment knobs (one
# kbench --phase indexless run per setting, stats first).
#   tools/gpu_r6_sdenv.sh <tag> "<ENV=..>" ...
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs HUFF_FIX_STATS=1 timeout -k 10 120 python tools/kbench.py --phase indexless --workload ${WL:-zipf} --iters 1 > /dev/null 2> $out/s$i.err || { tail -5 $out/s$i.err; exit 1; }
  env $envs timeout -k 10 120 python tools/kbench.py --phase indexless --workload ${WL:-zipf} --iters 20 > $out/k$i.json 2> $out/k$i.err || { tail -5 $out/k$i.err; exit 1; }
  echo "[$envs] $(grep 'sync decode' $out/s$i.err | tail -1) :: $(python3 -c "import json;print(round(json.load(open('$out/k$i.json'))['wall_ms_per_iter'],3))")"
done
