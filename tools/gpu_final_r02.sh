# Round-2 evidence: full GPU suite, smoke, every bench workload, rocprof kernel trace, PMC traffic + busy passes
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench_t16.json 2> $O/bench_t16.err || exit $?
head -c 300 $O/bench_t16.json; echo
for w in train s8 a64; do
  timeout -k 10 300 python -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-bs1 --no-secondary > $O/prof_bench.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --probe 0 --no-cpu-baseline --no-bs1 --no-secondary > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --probe 0 --no-cpu-baseline --no-bs1 --no-secondary > $O/pmc_write.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_busy -o run -- python3 $R/bench.py --steps 1 --warmup 1 --probe 0 --no-cpu-baseline --no-bs1 --no-secondary > $O/pmc_busy.log 2>&1 || exit $?
echo DONE
