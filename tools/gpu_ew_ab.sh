set -uo pipefail
out=gpurun_out/ew; mkdir -p $out
HUFF_LIB_AB=ew timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "test_device_job_medium" > $out/tests_ew.log 2>&1; echo "ew tests rc=$?: $(tail -1 $out/tests_ew.log)"
for rep in 1 2; do for w in zipf text; do for v in prod ew; do
  if [ $v = prod ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=ew; fi
  timeout -k 10 120 python tools/kbench.py --phase decode --workload $w --iters 20 > $out/${w}_${v}_$rep.json 2>>$out/err.log || exit 1
done; done; done
echo ew done
