# GDFN A/B: gdfn2 (opt-in, KDLAE_GDFN2=1, strip rows KDLAE_GDFN2_ROWS) vs r01's kernel
set -o pipefail
mkdir -p gpurun_out
KDLAE_GDFN2=1 timeout -k 10 300 python -u -m pytest tests/test_kdlae_gpu.py -k "golden or rand_512" -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_gdfn.log 2>&1 || { tail -30 gpurun_out/gputest_gdfn.log; exit 1; }
tail -1 gpurun_out/gputest_gdfn.log
for v in g2 g2r10 g2r4 g1; do
  unset KDLAE_GDFN2 KDLAE_GDFN2_ROWS
  [ $v != g1 ] && export KDLAE_GDFN2=1
  [ $v = g2r10 ] && export KDLAE_GDFN2_ROWS=10
  [ $v = g2r4 ] && export KDLAE_GDFN2_ROWS=4
  KDLAE_PROBE_DUMP=gpurun_out/probe_c3_$v.csv timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --probe 3 --no-cpu-baseline --no-bs1 > gpurun_out/probe_c3_$v.json 2> gpurun_out/probe_c3_$v.err || exit $?
done
echo DONE
