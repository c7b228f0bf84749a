# fused-FFN check: parity subset, then per-class probes with and without the fusion
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kdlae_gpu.py tests/test_baseline_batches_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_ffn.log 2>&1 || { tail -30 gpurun_out/gputest_ffn.log; exit 1; }
tail -1 gpurun_out/gputest_ffn.log
for v in fused unfused; do
  if [ $v = unfused ]; then export KDLAE_NO_FFN_FUSION=1; else unset KDLAE_NO_FFN_FUSION; fi
  for c in 1 3; do
    KDLAE_PROBE_DUMP=gpurun_out/probe_c${c}_$v.csv timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --probe $c --no-cpu-baseline --no-bs1 > gpurun_out/probe_c${c}_$v.json 2> gpurun_out/probe_c${c}_$v.err || exit $?
  done
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --probe 0 --no-cpu-baseline --no-bs1 > gpurun_out/bench_$v.json 2>&1 || exit $?
  head -c 180 gpurun_out/bench_$v.json; echo
done
