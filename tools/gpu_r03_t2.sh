# Round 3: training GEMM rework — training parity tests, launch trace, training bench
set -o pipefail
O=gpurun_out/${1:-t2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 300 --timeout-method thread > $O/gputest_train.log 2>&1 || { tail -40 $O/gputest_train.log; exit 1; }
tail -1 $O/gputest_train.log
timeout -k 10 300 python -u tools/train_trace.py $O/train_trace.csv > $O/train_trace.txt 2> $O/train_trace.err || { tail -20 $O/train_trace.err; exit 1; }
head -40 $O/train_trace.txt
timeout -k 10 300 python -u bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > $O/train_bench.json 2> $O/train_bench.err || { tail -20 $O/train_bench.err; exit 1; }
head -c 400 $O/train_bench.json
