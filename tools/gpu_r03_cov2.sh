# Round 3: which of libkdlae.so's kernels the GPU suite launches (rocprofv3 kernel trace, CSV).
# The multi-process test is left out under the profiler (its rank processes outlive the tracer's
# finalisation); its kernels are the single-process forward's.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-cov2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 1000 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u -m pytest $R/tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider --ignore=$R/tests/test_multiprocess_gpu.py > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
python3 $R/tools/kernel_coverage.py $O/prof > $O/coverage.txt; head -1 $O/coverage.txt
rm -f $O/prof/*kernel_trace.csv
