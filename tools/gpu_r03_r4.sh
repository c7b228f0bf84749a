# Round 3: K = 48 resident GEMMs at 4 waves/SIMD with the unit-major body (KDLAE_RES4_K48 build) vs default
set -o pipefail
O=gpurun_out/r4
mkdir -p $O
L=rethink_acoustic_image_enhancement_amd
timeout -k 10 200 python -u tools/out_hash.py > $O/hash_base.json 2> $O/hash_base.err || exit $?
KDLAE_LIB=$GRAFT_REPO_ROOT/$L/libkdlae_r4.so timeout -k 10 200 python -u tools/out_hash.py > $O/hash_r4.json 2> $O/hash_r4.err || exit $?
cat $O/hash_base.json $O/hash_r4.json
VARIANTS="base=default r4=$L/libkdlae_r4.so base2=default r42=$L/libkdlae_r4.so" PROBE=1 bash tools/gpu_ab.sh || exit $?
rm -rf $O/ab; cp -r gpurun_out/ab $O/ab; rm -rf gpurun_out/ab
