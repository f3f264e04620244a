#!/usr/bin/env bash
# Round 6: the GPU suite, then the default bench line and the strong-scaling
# N=1 records at the 8/4/2-rank shard sizes (128/256/512 MiB).
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r6check}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], {k: v['avg_ms'] for k, v in d['kernels'].items()}); print('zipf', d['side']['zipf']['value'], d['side']['zipf']['e2e']['indexfree_decode_ms'], {k: v['avg_ms'] for k, v in d['side']['zipf']['kernels'].items()}); print('general', d['general']['value'], {k: v['avg_ms'] for k, v in d['general']['kernels'].items()})" $out/bench.json
for mb in 128 256 512; do
  timeout -k 10 200 python -u bench.py --scaling strong --total-bytes $((mb << 20)) --side none --no-general --file-path none --no-cpu-baseline --no-other-scaling --steps 20 --warmup 3 > $out/strong_$mb.json 2> $out/strong_$mb.err || { tail -5 $out/strong_$mb.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print('strong', sys.argv[2], d['value'], d['ms_per_step'], d.get('host_gap_ms'), {k: v['avg_ms'] for k, v in d['kernels'].items()})" $out/strong_$mb.json $mb
done
