# Fused attention output + LN + project_in (C = 48): parity suite, class-1 probe fused vs unfused, bench
set -o pipefail
mkdir -p gpurun_out/ai
timeout -k 10 600 python -u -m pytest tests/test_kdlae_gpu.py tests/test_baseline_batches_gpu.py tests/test_checkpoint_gpu.py -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/ai/gputest.log 2>&1 || { tail -40 gpurun_out/ai/gputest.log; exit 1; }
tail -1 gpurun_out/ai/gputest.log
for v in fused unfused; do
  if [ $v = unfused ]; then export KDLAE_NO_ATTN_IN_FUSION=1; fi
  KDLAE_PROBE_DUMP=gpurun_out/ai/probe_c1_$v.csv timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --probe 1 --no-cpu-baseline --no-bs1 > gpurun_out/ai/$v.json 2> gpurun_out/ai/$v.err || exit $?
  python tools/probe_table.py gpurun_out/ai/probe_c1_$v.csv > gpurun_out/ai/probe_c1_$v.txt
  head -14 gpurun_out/ai/probe_c1_$v.txt
done
unset KDLAE_NO_ATTN_IN_FUSION
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ai/bench_t16.json 2> gpurun_out/ai/bench_t16.err || exit $?
head -c 300 gpurun_out/ai/bench_t16.json; echo
echo DONE
