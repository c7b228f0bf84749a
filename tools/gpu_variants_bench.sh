# A/B of prebuilt library variants on one bench workload: VARIANTS="a b" WL=train
set -o pipefail
mkdir -p gpurun_out
L=rethink_acoustic_image_enhancement_amd/libkdlae.so
for v in $VARIANTS; do
  cp scratch/libkdlae_$v.so $L
  timeout -k 10 200 python -u bench.py --workload ${WL:-train} --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/vb_$v.json 2> gpurun_out/vb_$v.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/vb_$v.json')); print('$v', d['value'], d['ms_per_step'])"
done
