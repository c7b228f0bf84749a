# Resident GEMM: waves 4-7 start late (s_sleep 40 / 127 x 64 cycles) vs the in-tree build (class-1 probe)
set -o pipefail
mkdir -p gpurun_out/stag
for v in base st40 st127 base2; do
  if [ $v = base ] || [ $v = base2 ]; then unset KDLAE_LIB; else export KDLAE_LIB=$PWD/rethink_acoustic_image_enhancement_amd/libkdlae_$v.so; fi
  KDLAE_PROBE_DUMP=gpurun_out/stag/probe_c1_$v.csv timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --probe 1 --no-cpu-baseline --no-bs1 --no-secondary > gpurun_out/stag/$v.json 2> gpurun_out/stag/$v.err || exit $?
  python tools/probe_table.py gpurun_out/stag/probe_c1_$v.csv | head -9
done
echo DONE
