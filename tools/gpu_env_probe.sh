# per-launch probe of one kernel class under an env toggle: ENVSET="VAR=val" CLS=2 NAME=x
set -o pipefail
mkdir -p gpurun_out
env $ENVSET KDLAE_PROBE_DUMP=gpurun_out/probe_$NAME.csv timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --probe $CLS --no-cpu-baseline > gpurun_out/probe_$NAME.json 2> gpurun_out/probe_$NAME.err
