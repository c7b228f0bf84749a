# A/B of training-step library builds: launch trace + training bench per variant.
# usage: bash tools/gpu_ab_train.sh <outdir> <variant>...   (variant "base" = the default libkdlae.so,
# else rethink_acoustic_image_enhancement_amd/libkdlae_<variant>.so)
set -o pipefail
R=$GRAFT_REPO_ROOT
L=$R/rethink_acoustic_image_enhancement_amd
O=$R/gpurun_out/$1
shift
mkdir -p $O
cd $R
for v in "$@"; do
  if [ $v = base ]; then unset KDLAE_LIB; else export KDLAE_LIB=$L/libkdlae_$v.so; fi
  timeout -k 10 300 python -u tools/train_trace.py $O/$v.csv > $O/$v.txt 2> $O/$v.err || { tail -20 $O/$v.err; exit 1; }
  echo "$v: $(head -1 $O/$v.txt); conv3 $(grep -E 'fwd3|dX3|dW3' $O/$v.txt | awk '{s+=$4} END {print s}') ms"
  timeout -k 10 300 python -u bench.py --workload train --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  echo "$v bench: $(python3 -c "import json,sys; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
