# Per-layer time vs batch size: does a layer get faster per pixel when its intermediate fits the
# 256 MiB Infinity Cache (bs=1: C96@256^2 project_in output = 134 MB; bs=16: 2.1 GB)?
set -o pipefail
mkdir -p gpurun_out/mall
for B in 1 4 16; do
  for c in 1 3; do
    KDLAE_PROBE_DUMP=gpurun_out/mall/probe_c${c}_b$B.csv timeout -k 10 200 python -u bench.py --batch $B --steps 2 --warmup 1 --probe $c --no-cpu-baseline --no-bs1 --no-secondary > gpurun_out/mall/b${B}_c$c.json 2> gpurun_out/mall/b${B}_c$c.err || exit $?
  done
done
echo DONE
