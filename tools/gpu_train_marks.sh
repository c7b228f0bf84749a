# Marked backward + bucketed DDP all-reduce: GPU tests, then the training bench (N=1 path unchanged)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_multiprocess_gpu.py -x -v -rP --timeout 300 --timeout-method thread > gpurun_out/gputest_marks.log 2>&1 || { tail -40 gpurun_out/gputest_marks.log; exit 1; }
grep -E "gradient-ready|gradient buckets|passed|failed" gpurun_out/gputest_marks.log | tail -8
timeout -k 10 300 python -u bench.py --workload train --no-cpu-baseline > gpurun_out/bench_train_marks.json 2> gpurun_out/bench_train_marks.err || exit $?
head -c 400 gpurun_out/bench_train_marks.json; echo
echo DONE
