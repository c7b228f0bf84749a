# Round 3: Gram sweep A/B (class 2) and GEMM ablations (class 1: no stores / no A loads, timing only)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ab2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py tests/test_graph_gpu.py -m gpu -v -rP --timeout 200 --timeout-method thread > $O/gputest.log 2>&1; tail -1 $O/gputest.log
L=rethink_acoustic_image_enhancement_amd
VARIANTS="base=default g9=$L/libkdlae_g9.so r10=$L/libkdlae_r10.so r9=$L/libkdlae_r9.so base2=default" PROBE=2 bash tools/gpu_ab.sh || exit $?
rm -rf $O/gram; cp -r gpurun_out/ab $O/gram; rm -rf gpurun_out/ab
VARIANTS="base=default nost=$L/libkdlae_nost.so nold=$L/libkdlae_nold.so" PROBE=1 bash tools/gpu_ab.sh || exit $?
rm -rf $O/gemm; cp -r gpurun_out/ab $O/gemm; rm -rf gpurun_out/ab
timeout -k 10 300 python -u tools/micro/blas_shapes.py > $O/blas_shapes.jsonl 2> $O/blas_shapes.err || exit $?
tail -2 $O/blas_shapes.err
