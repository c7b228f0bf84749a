set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train -o run -- python3 $R/bench.py --workload train --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_train.log 2>&1
