# Round 3: kernel-variant tests, then the whole GPU suite (one process each), logs under gpurun_out/$1
set -o pipefail
O=gpurun_out/${1:-suite}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernel_variants_infer_gpu.py tests/test_kernel_variants_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/variants.log 2>&1 || { tail -40 $O/variants.log; exit 1; }
tail -2 $O/variants.log
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_kernel_variants_infer_gpu.py --deselect tests/test_kernel_variants_gpu.py > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
