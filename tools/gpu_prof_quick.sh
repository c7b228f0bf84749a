# Kernel-trace summary of the default bench (5 timed steps)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/profq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-bs1 --no-secondary > $O/prof_bench.log 2>&1 || exit $?
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
echo DONE
