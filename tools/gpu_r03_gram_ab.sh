# Round 3: Gram sweep A/B (probe class 2 per variant): 10 vs 9 waves at Ch = 96, rolling stencil window
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-grab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py tests/test_graph_gpu.py -m gpu -v -rP --timeout 200 --timeout-method thread > $O/gputest.log 2>&1; tail -1 $O/gputest.log
L=rethink_acoustic_image_enhancement_amd
export VARIANTS="base=default g9=$L/libkdlae_g9.so r10=$L/libkdlae_r10.so r9=$L/libkdlae_r9.so base2=default"
PROBE=2 bash tools/gpu_ab.sh
cp -r gpurun_out/ab $O/ab
