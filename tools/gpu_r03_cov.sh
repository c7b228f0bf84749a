# Round-3: the whole GPU suite under a rocprofv3 kernel trace (which kernels each test run launches:
# coverage of every kernel libkdlae.so can launch), smoke, then the default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-cov}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 1000 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u -m pytest $R/tests -m gpu -v -rP --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; }
tail -1 $O/gputest.log
grep "t_mdd_512" $O/gputest.log | head -4
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
head -c 600 $O/bench.json; echo
