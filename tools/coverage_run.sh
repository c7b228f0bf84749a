#!/bin/bash
# Kernel coverage of the GPU suite: rocprofv3 kernel trace of `pytest -m gpu` (CSV output, a progress
# line every 30 s while the profiler writes its trace) -> tools/kernel_coverage.py -> gpurun_out/r6w/.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6w; mkdir -p $O && cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/cov -o run -- python3 -u -m pytest $R/tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 30; echo "[progress] $(date +%T) suite.log $(wc -c < $O/suite.log) B"; done
wait $pid || exit $?
cd $R && python3 tools/kernel_coverage.py /tmp/cov > $O/coverage.txt 2>&1
tail -2 $O/suite.log; tail -6 $O/coverage.txt
