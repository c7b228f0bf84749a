# State check: full GPU suite (printed parity numbers), smoke, default bench, kernel-trace summary
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/state
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench_t16.json 2> $O/bench_t16.err || exit $?
head -c 800 $O/bench_t16.json; echo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-bs1 --no-secondary > $O/prof_bench.log 2>&1 || exit $?
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
echo DONE
