# Round 3: narrow-channel training convs — launch trace + training bench, then the kernel-coverage trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-t3}
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/train_trace.py $O/train_trace.csv > $O/train_trace.txt 2> $O/train_trace.err || { tail -20 $O/train_trace.err; exit 1; }
head -12 $O/train_trace.txt
timeout -k 10 300 python -u bench.py --workload train --steps 20 --warmup 5 --no-cpu-baseline > $O/train_bench.json 2> $O/train_bench.err || { tail -20 $O/train_bench.err; exit 1; }
head -c 300 $O/train_bench.json; echo
bash tools/gpu_r03_cov2.sh ${1:-t3}/cov
