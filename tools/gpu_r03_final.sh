# Round 3 final: whole GPU suite, smoke(), default bench line (T16 + S8/A64 extras + CPU baseline)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-final}
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
head -c 500 $O/bench.json; echo
