# MFMA / VALU busy per kernel class (one --pmc pass each, kernel-trace-free), plus the MFMA peak micro
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/tools/micro/mfma_peak > $O/mfma_peak.txt 2>&1 || exit $?
cat $O/mfma_peak.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/micro -o run -- $R/tools/micro/mfma_peak > $O/micro.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/t16 -o run -- python3 $R/bench.py --steps 1 --warmup 1 --probe 0 --no-cpu-baseline --no-bs1 --no-secondary > $O/t16.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc MfmaUtil VALUBusy --output-format csv -d $O/t16_derived -o run -- python3 $R/bench.py --steps 1 --warmup 1 --probe 0 --no-cpu-baseline --no-bs1 --no-secondary > $O/t16_derived.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_LDS_ADDR_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/t16_lds -o run -- python3 $R/bench.py --steps 1 --warmup 1 --probe 0 --no-cpu-baseline --no-bs1 --no-secondary > $O/t16_lds.log 2>&1 || exit $?
ls -R $O | head -30
