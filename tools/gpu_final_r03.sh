# Round-3 evidence, part A: full GPU suite (as the driver runs it), smoke, every bench workload
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-final3}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench_t16.json 2> $O/bench_t16.err || exit $?
head -c 400 $O/bench_t16.json; echo
for w in train s8 a64; do
  timeout -k 10 300 python -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || exit $?
  head -c 200 $O/bench_$w.json; echo
done
