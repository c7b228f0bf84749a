set -o pipefail
L=rethink_acoustic_image_enhancement_amd
mkdir -p gpurun_out/dwab
for v in base u8 ty32 u2; do
  if [ $v = base ]; then unset KDLAE_LIB; else export KDLAE_LIB=$GRAFT_REPO_ROOT/$L/libkdlae_$v.so; fi
  timeout -k 10 200 python -u tools/train_trace.py gpurun_out/dwab/$v.csv > gpurun_out/dwab/$v.txt 2> gpurun_out/dwab/$v.err || exit 1
  echo "$v: $(head -1 gpurun_out/dwab/$v.txt) $(grep -E 'dwgate|dw_bwd' gpurun_out/dwab/$v.txt | awk '{s+=$3} END {print s}') ms dw"
done
