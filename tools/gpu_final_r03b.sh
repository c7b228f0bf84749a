# Round-3 evidence, part B: rocprofv3 kernel traces (T16 bench, training step), PMC traffic + busy
# passes (one counter group per run, kernel-trace free), per the MI355X guide's HBM recipe
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-final3b}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-bs1 --no-secondary > $O/prof_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_train -o run -- python3 $R/bench.py --workload train --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_train.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --probe 0 --no-cpu-baseline --no-bs1 --no-secondary > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --probe 0 --no-cpu-baseline --no-bs1 --no-secondary > $O/pmc_write.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_busy -o run -- python3 $R/bench.py --steps 1 --warmup 1 --probe 0 --no-cpu-baseline --no-bs1 --no-secondary > $O/pmc_busy.log 2>&1 || exit $?
echo DONE
