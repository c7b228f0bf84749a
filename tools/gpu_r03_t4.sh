# Round 3: depthwise one-row-ahead prefetch A/B (KDLAE_DWG_PF) + dW3-small rework: training parity on
# the default library, then launch traces and training benches of both libraries
set -o pipefail
R=$GRAFT_REPO_ROOT
L=$R/rethink_acoustic_image_enhancement_amd
O=$R/gpurun_out/${1:-t4}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest_train.log 2>&1 || { tail -40 $O/gputest_train.log; exit 1; }
tail -1 $O/gputest_train.log
for v in base pf; do
  if [ $v = base ]; then unset KDLAE_LIB; else export KDLAE_LIB=$L/libkdlae_$v.so; fi
  timeout -k 10 300 python -u tools/train_trace.py $O/$v.csv > $O/$v.txt 2> $O/$v.err || { tail -20 $O/$v.err; exit 1; }
  echo "$v: $(head -1 $O/$v.txt) $(grep -E 'dwgate|dw_bwd' $O/$v.txt | awk '{s+=$3} END {print s}') ms dw; $(grep dw3_small $O/$v.txt)"
  timeout -k 10 300 python -u bench.py --workload train --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  echo "$v bench: $(head -c 220 $O/bench_$v.json)"
done
