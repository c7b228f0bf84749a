set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gputest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_t16.json 2> gpurun_out/bench_t16.err && \
timeout -k 10 200 python -u bench.py --workload train --no-cpu-baseline > gpurun_out/bench_train.json 2> gpurun_out/bench_train.err && \
timeout -k 10 200 python -u bench.py --workload s8 --no-cpu-baseline > gpurun_out/bench_s8.json 2> gpurun_out/bench_s8.err && \
timeout -k 10 200 python -u bench.py --workload a64 --no-cpu-baseline > gpurun_out/bench_a64.json 2> gpurun_out/bench_a64.err && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_bench.log 2>&1
