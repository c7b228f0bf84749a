# GDFN C = 48: 16x12 tiles (KDLAE_GDFN_TILE=7) vs the default 16x8, same run; parity first
set -o pipefail
mkdir -p gpurun_out/t7
KDLAE_GDFN_TILE=7 timeout -k 10 300 python -u -m pytest tests/test_kdlae_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t7/gputest.log 2>&1 || { tail -30 gpurun_out/t7/gputest.log; exit 1; }
tail -1 gpurun_out/t7/gputest.log
for v in t1 t7 t1b t7b; do
  export KDLAE_GDFN_TILE=${v:1:1}
  KDLAE_PROBE_DUMP=gpurun_out/t7/probe_c3_$v.csv timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --probe 3 --no-cpu-baseline --no-bs1 > gpurun_out/t7/$v.json 2> gpurun_out/t7/$v.err || exit $?
  python tools/probe_table.py gpurun_out/t7/probe_c3_$v.csv > gpurun_out/t7/probe_c3_$v.txt
  head -5 gpurun_out/t7/probe_c3_$v.txt
done
echo DONE
