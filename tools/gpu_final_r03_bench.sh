# Round-3 evidence: every bench workload (default T16 line with CPU baseline, then train / S8 / A64)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-final3}
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench_t16.json 2> $O/bench_t16.err || { tail -5 $O/bench_t16.err; exit 1; }
head -c 400 $O/bench_t16.json; echo
for w in train s8 a64; do
  timeout -k 10 300 python -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail -5 $O/bench_$w.err; exit 1; }
  head -c 200 $O/bench_$w.json; echo
done
