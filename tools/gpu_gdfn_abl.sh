# GDFN ablations (timing only, outputs wrong): 1 = every tile's halo from tile (0,0) (L2-hot),
# 2 = no MFMA (gate only), 3 = no stencil/GELU (DMA + MFMA only)
set -o pipefail
mkdir -p gpurun_out/abl
for v in 1 2 3; do
  KDLAE_LIB=$PWD/rethink_acoustic_image_enhancement_amd/libkdlae_abl$v.so KDLAE_PROBE_DUMP=gpurun_out/abl/probe_c3_abl$v.csv timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --probe 3 --no-cpu-baseline --no-bs1 --no-secondary > gpurun_out/abl/abl$v.json 2> gpurun_out/abl/abl$v.err || exit $?
  python tools/probe_table.py gpurun_out/abl/probe_c3_abl$v.csv | head -5
done
echo DONE
