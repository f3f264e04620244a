#!/usr/bin/env bash
# One GPU-box session for the round's artifacts: parity tests, rocprofv3
# profiles (kernel trace + separate PMC passes) per workload turned into
# profiles/traffic_<w>.json, then the N=1 bench lines (with cpu_baseline) and a
# 2-rank rehearsal of the N>1 path (gloo, both ranks on the one GPU).
#   tools/gpu_round.sh <tag> [skip-tests]
set -euo pipefail
tag=${1:-dev}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
out=gpurun_out/$tag
mkdir -p "$out"
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$out/gpu_tests.log" 2>&1
fi
for w in uniform zipf text; do
  bash tools/profile.sh all $w "${tag}_all_$w" > /dev/null
  python tools/summarize_prof.py "gpurun_out/prof/${tag}_all_$w" > "$out/prof_all_$w.json"
  python tools/make_traffic.py "$out/prof_all_$w.json" $w > /dev/null
  cp "gpurun_out/prof/${tag}_all_$w/trace/run_kernel_stats.csv" "$out/kernel_stats_all_$w.csv"
done
for w in uniform zipf text; do
  timeout -k 10 400 python bench.py --workload $w > "$out/bench_$w.json" 2> "$out/bench_$w.err"
done
HUFF_DISABLE_FIXED8=1 timeout -k 10 300 python bench.py --no-cpu-baseline > "$out/bench_uniform_general.json" 2> "$out/bench_uniform_general.err"
# the per-GPU shard sizes of BASELINE configs[3] (16 GiB / 8) and configs[4] (64 GiB / 8)
timeout -k 10 300 python bench.py --no-cpu-baseline --bytes-per-gpu $((2<<30)) > "$out/bench_uniform_2GiB.json" 2> "$out/bench_uniform_2GiB.err"
timeout -k 10 400 python bench.py --no-cpu-baseline --workload text --steps 5 --warmup 2 --bytes-per-gpu $((8<<30)) > "$out/bench_text_8GiB.json" 2> "$out/bench_text_8GiB.err"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --workload text --bytes-per-gpu $((1<<28)) \
  --dist-backend gloo > "$out/bench_2rank_gloo.json" 2> "$out/bench_2rank_gloo.err"
# wider letters: timings at 1 GiB and a kernel-trace profile
for w in 2 4 8; do
  timeout -k 10 300 python tools/wbench.py --width $w --indexless > "$out/wide_w$w.json" 2> "$out/wide_w$w.err"
done
bash tools/prof_wide.sh 2 "${tag}_wide_w2" > /dev/null
python tools/summarize_prof.py "gpurun_out/prof/${tag}_wide_w2" > "$out/prof_wide_w2.json"
cp "gpurun_out/prof/${tag}_wide_w2/trace/run_kernel_stats.csv" "$out/kernel_stats_wide_w2.csv"
mkdir -p "$out/profiles_copy" && cp profiles/traffic_*.json "$out/profiles_copy/"
echo "gpu_round $tag done"
