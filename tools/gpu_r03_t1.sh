# Round 3: parity of the default library + output digests + training-step launch trace
set -o pipefail
O=gpurun_out/t1
mkdir -p $O
timeout -k 10 200 python -u tools/out_hash.py > $O/hash.json 2> $O/hash.err || exit $?
cat $O/hash.json
timeout -k 10 500 python -u -m pytest tests/test_kdlae_gpu.py tests/test_baseline_batches_gpu.py -x -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python -u tools/train_trace.py $O/train_trace.csv > $O/train_trace.txt 2> $O/train_trace.err || { tail -20 $O/train_trace.err; exit 1; }
head -60 $O/train_trace.txt
