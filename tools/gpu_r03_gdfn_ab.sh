# Round 3: quick parity of the changed tests, then the GDFN scheduling A/B (probe class 3 per variant)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-gab}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kdlae_gpu.py::test_mdd_512_config1 "tests/test_train_gpu.py::test_mark_events_fire_after_their_suffix_is_final" tests/test_graph_gpu.py -m gpu -v -rP --timeout 200 --timeout-method thread > $O/gputest.log 2>&1; tail -1 $O/gputest.log
grep "t_mdd_512\|marks, snap" $O/gputest.log
export VARIANTS="base=default sgb1=rethink_acoustic_image_enhancement_amd/libkdlae_sgb1.so sgb2=rethink_acoustic_image_enhancement_amd/libkdlae_sgb2.so sgb3=rethink_acoustic_image_enhancement_amd/libkdlae_sgb3.so noslp=rethink_acoustic_image_enhancement_amd/libkdlae_noslp.so"
PROBE=3 bash tools/gpu_ab.sh
cp -r gpurun_out/ab $O/ab
