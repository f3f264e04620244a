#!/usr/bin/env bash
# decode timing A/B over env settings (each arg: NAME=a,VAR=b,...), zipf + text, interleaved twice
set -uo pipefail
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
for rep in 1 2; do
  for w in zipf text; do
    for cfg in "$@"; do
      name=${cfg%%=*}; envs=${cfg#*=}
      env $(echo "$envs" | tr ',' ' ') timeout -k 10 120 python tools/kbench.py --phase decode --workload $w --iters 20 >> $out/${w}_$name.json 2>> $out/err.log || exit 1
    done
  done
done
echo "dec_ab $tag done"
