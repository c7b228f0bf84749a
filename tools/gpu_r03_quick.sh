# Round-3 quick check: the T-path GPU parity file(s) given, then the default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-quick}
shift
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${@:-tests/test_kdlae_gpu.py} -m gpu -x -v -rP --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
grep "t_mdd_512" $O/gputest.log | head -4
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
head -c 600 $O/bench.json; echo
