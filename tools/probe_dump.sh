set -o pipefail
mkdir -p gpurun_out
for c in 1 2 3; do
  KDLAE_PROBE_DUMP=gpurun_out/probe_c$c.csv timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --probe $c --no-cpu-baseline > gpurun_out/probe_c$c.json 2> gpurun_out/probe_c$c.err || exit $?
done
