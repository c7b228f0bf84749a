set -o pipefail
mkdir -p gpurun_out
KDLAE_GEMM_WPE=4 KDLAE_PROBE_DUMP=gpurun_out/probe_wpe4.csv timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --probe 1 --no-cpu-baseline > gpurun_out/probe_wpe4.json 2> gpurun_out/probe_wpe4.err
