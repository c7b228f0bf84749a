# GDFN A/B: r01 kernel tile variants (KDLAE_GDFN_TILE 0/1/2) and gdfn2 (KDLAE_GDFN2=1)
set -o pipefail
mkdir -p gpurun_out
for t in 2 3; do
  KDLAE_GDFN_TILE=$t timeout -k 10 300 python -u -m pytest tests/test_kdlae_gpu.py -k "golden or rand_512" -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_gdfn_t$t.log 2>&1 || { tail -30 gpurun_out/gputest_gdfn_t$t.log; exit 1; }
  tail -1 gpurun_out/gputest_gdfn_t$t.log
done
for v in t1 t2 t3 t0; do
  export KDLAE_GDFN_TILE=${v#t}
  KDLAE_PROBE_DUMP=gpurun_out/probe_c3_$v.csv timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --probe 3 --no-cpu-baseline --no-bs1 > gpurun_out/probe_c3_$v.json 2> gpurun_out/probe_c3_$v.err || exit $?
done
echo DONE
