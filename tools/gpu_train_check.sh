set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { tail -30 gpurun_out/gputest.log; exit 1; }
tail -1 gpurun_out/gputest.log
timeout -k 10 200 python -u bench.py --workload train --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/tlog.json 2> gpurun_out/tlog.err || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload train > gpurun_out/bench_train.json 2> gpurun_out/bench_train.err || exit $?
head -c 300 gpurun_out/bench_train.json; echo
python -c "import json; d=json.load(open('gpurun_out/bench_train.json')); print(d.get('parity'))"
