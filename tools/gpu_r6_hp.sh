#!/usr/bin/env bash
# Round 6: the persistent pass 1 (k_hist1x2p, HUFF_LIB_AB=persist) against the
# one-shot k_hist1x2: its parity tests, then kbench --phase hist and the
# headline bench, alternated.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r6hp}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
HUFF_LIB_AB=persist timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "weights or pass1 or hist or one_call or pipelined or full_size" > $out/pytest.log 2>&1; tail -2 $out/pytest.log
B="--side none --no-general --file-path none --no-cpu-baseline --no-other-scaling --steps 20 --warmup 3"
for r in 1 2; do
  for v in default persist; do
    if [ $v = default ]; then env=""; else env="HUFF_LIB_AB=$v"; fi
    for wl in uniform zipf; do
      env $env timeout -k 10 120 python -u tools/kbench.py --phase hist --workload $wl --iters 20 > $out/hist_${v}_${wl}_$r.json 2> $out/hist_${v}_${wl}_$r.err || { tail -5 $out/hist_${v}_${wl}_$r.err; exit 1; }
    done
    env $env timeout -k 10 200 python -u bench.py $B > $out/bench_${v}_$r.json 2> $out/bench_${v}_$r.err || { tail -5 $out/bench_${v}_$r.err; exit 1; }
  done
done
grep -H hist_ms $out/hist_*.json | sed "s|$out/||"
for f in $out/bench_*.json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})" $f; done
cd /tmp && export TMPDIR=/tmp
HUFF_LIB_AB=persist timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 $root/tools/kbench.py --phase hist --workload uniform --iters 20 > $out/prof.log 2>&1 || { tail -5 $out/prof.log; exit 1; }
grep -h "k_hist\|k_rows" $out/prof/run_kernel_stats.csv | cut -c1-150
