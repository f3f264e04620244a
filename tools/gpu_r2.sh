#!/usr/bin/env bash
# Round-2 GPU session: parity suite, bench lines (N=1 with the configs[2] side
# result, strong-scaling mode, a 2-rank gloo rehearsal of the N>1 path).
#   tools/gpu_r2.sh <tag> [tests|bench|all]
set -uo pipefail
tag=${1:-dev}; what=${2:-all}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root"
out=gpurun_out/$tag
mkdir -p "$out"
if [ "$what" = tests ] || [ "$what" = all ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$out/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$out/gpu_tests.log"; exit 1; }
  tail -3 "$out/gpu_tests.log"
fi
if [ "$what" = bench ] || [ "$what" = all ]; then
  timeout -k 10 400 python bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; tail -20 "$out/bench.err"; exit 1; }
  timeout -k 10 300 python bench.py --scaling strong --side none --no-cpu-baseline > "$out/bench_strong1.json" 2> "$out/bench_strong1.err" || { echo "strong bench failed"; tail -20 "$out/bench_strong1.err"; exit 1; }
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --workload text --bytes-per-gpu $((1<<28)) \
    --dist-backend gloo --side none > "$out/bench_2rank_gloo.json" 2> "$out/bench_2rank_gloo.err" || { echo "2-rank failed"; tail -20 "$out/bench_2rank_gloo.err"; exit 1; }
fi
echo "gpu_r2 $tag done"
