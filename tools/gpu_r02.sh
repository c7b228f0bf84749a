# r02 check: env probe, full GPU suite (with the tests' printed parity numbers), default bench
set -o pipefail
mkdir -p gpurun_out
{ cat /sys/fs/cgroup/cpu.max 2>&1; nproc; python -c "import os; print(os.cpu_count(), len(os.sched_getaffinity(0)))"; echo "OMP=$OMP_NUM_THREADS"; } > gpurun_out/env.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_t16.json 2> gpurun_out/bench_t16.err || exit $?
head -c 600 gpurun_out/bench_t16.json; echo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/rocprof_counters.txt 2>&1 || true
