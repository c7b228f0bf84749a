# quick GPU check: parity suite, headline bench, per-launch GEMM probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { tail -30 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_t16.json 2> gpurun_out/bench_t16.err || exit $?
cat gpurun_out/bench_t16.json | head -c 400; echo
for w in ${EXTRA_WL:-}; do
  timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || exit $?
  head -c 200 gpurun_out/bench_$w.json; echo
done
for c in ${PROBES:-1}; do
  KDLAE_PROBE_DUMP=gpurun_out/probe_c$c.csv timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --probe $c --no-cpu-baseline > gpurun_out/probe_c$c.json 2> gpurun_out/probe_c$c.err || exit $?
done
