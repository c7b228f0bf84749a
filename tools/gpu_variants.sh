# A/B of prebuilt library variants: VARIANTS="w9 w10" CLS=2 (each: GPU parity suite + per-launch probe)
set -o pipefail
mkdir -p gpurun_out
L=rethink_acoustic_image_enhancement_amd/libkdlae.so
cp $L gpurun_out/libkdlae.orig.so
for v in $VARIANTS; do
  cp scratch/libkdlae_$v.so $L
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_$v.log 2>&1 || { tail -20 gpurun_out/gputest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/gputest_$v.log)"
  KDLAE_PROBE_DUMP=gpurun_out/probe_$v.csv timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --probe ${CLS:-2} --no-cpu-baseline > gpurun_out/probe_$v.json 2> gpurun_out/probe_$v.err || exit $?
done
rm gpurun_out/libkdlae.orig.so
