#!/usr/bin/env bash
# Round 6: the strong-scaling curve's per-rank sizes measured on ONE GPU
# (VERDICT r5 item 4): bench.py at N = 1 with --scaling strong and
# --total-bytes = 1 GiB / N for N = 8, 4, 2, 1 (128 / 256 / 512 / 1024 MiB per
# rank), plus a kernel trace of the 128 MiB step.
#   tools/gpu_r6_scale.sh <tag>
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r6scale}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
for mib in 128 256 512 1024; do
  timeout -k 10 200 python -u bench.py --scaling strong --total-bytes $((mib << 20)) --side none --no-general \
    --file-path none --no-cpu-baseline --no-other-scaling --steps 20 --warmup 5 > $out/strong_${mib}.json 2> $out/strong_${mib}.err \
    || { tail -20 $out/strong_${mib}.err; exit 1; }
  echo "strong $mib MiB done"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/trace128 -o run --output-format csv -- python3 $root/bench.py \
  --scaling strong --total-bytes $((128 << 20)) --side none --no-general --file-path none --no-cpu-baseline \
  --no-other-scaling --steps 10 --warmup 3 > $out/trace128.log 2>&1 || { tail -20 $out/trace128.log; exit 1; }
echo "trace done"
