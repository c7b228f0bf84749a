# chunked-GEMM A/B: parity subset, then per-launch GEMM probe with the r01 chunked kernel and the r02 one
set -o pipefail
mkdir -p gpurun_out
export KDLAE_NO_FFN_FUSION=1
timeout -k 10 600 python -u -m pytest tests/test_kdlae_gpu.py tests/test_baseline_batches_gpu.py tests/test_kdlae_s_gpu.py tests/test_asdqe_gpu.py tests/test_checkpoint_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_ab.log 2>&1 || { tail -30 gpurun_out/gputest_ab.log; exit 1; }
tail -1 gpurun_out/gputest_ab.log
for v in chunk2 chunk1; do
  if [ $v = chunk1 ]; then export KDLAE_GEMM_CHUNK1=1; else unset KDLAE_GEMM_CHUNK1; fi
  KDLAE_PROBE_DUMP=gpurun_out/probe_c1_$v.csv timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --probe 1 --no-cpu-baseline --no-bs1 > gpurun_out/probe_c1_$v.json 2> gpurun_out/probe_c1_$v.err || exit $?
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --probe 0 --no-cpu-baseline --no-bs1 > gpurun_out/bench_$v.json 2>&1 || exit $?
  head -c 180 gpurun_out/bench_$v.json; echo
  for w in s8 a64; do
    timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_${w}_$v.json 2>&1 || exit $?
    head -c 150 gpurun_out/bench_${w}_$v.json; echo
  done
done
