# Round 3 final training evidence: parity, launch trace, bench line, rocprofv3 kernel summary
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-t5}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_kernel_variants_infer_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest_train.log 2>&1 || { tail -40 $O/gputest_train.log; exit 1; }
tail -1 $O/gputest_train.log
timeout -k 10 300 python -u tools/train_trace.py $O/trace.csv > $O/trace.txt 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
head -1 $O/trace.txt
timeout -k 10 300 python -u bench.py --workload train --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_train.json 2> $O/bench_train.err || { tail -20 $O/bench_train.err; exit 1; }
head -c 260 $O/bench_train.json; echo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 $R/bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
cd $R && python3 tools/prof_summary.py $(ls $O/kt/*/run_results.db $O/kt/run_results.db 2>/dev/null | head -1) --per 12 > $O/train_summary.txt 2>&1; head -5 $O/train_summary.txt; tail -1 $O/train_summary.txt
