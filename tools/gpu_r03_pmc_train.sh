# Round 3: PMC passes over one training step (wave-state split, VALU / VMEM issue, TA busy, L2 hit)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-pmc_train}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 $R/bench.py --workload train --steps 1 --warmup 1 --no-cpu-baseline > $O/p1.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc TA_TA_BUSY_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 $R/bench.py --workload train --steps 1 --warmup 1 --no-cpu-baseline > $O/p2.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o run -- python3 $R/bench.py --workload train --steps 1 --warmup 1 --no-cpu-baseline > $O/p3.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p4 -o run -- python3 $R/bench.py --workload train --steps 1 --warmup 1 --no-cpu-baseline > $O/p4.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt -o run -- python3 $R/bench.py --workload train --steps 1 --warmup 1 --no-cpu-baseline > $O/kt.log 2>&1 || exit $?
echo DONE
