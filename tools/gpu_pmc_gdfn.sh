# GDFN PMC: busy/wait split and memory-path counters for gdfn2 (default) and r01's kernel (KDLAE_GDFN1)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcg
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in g2; do
  unset KDLAE_GDFN2; [ $v = g2 ] && export KDLAE_GDFN2=1
  timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/busy_$v -o run -- python3 $R/bench.py --steps 1 --warmup 0 --probe 0 --no-cpu-baseline --no-bs1 > $O/busy_$v.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $O/mem_$v -o run -- python3 $R/bench.py --steps 1 --warmup 0 --probe 0 --no-cpu-baseline --no-bs1 > $O/mem_$v.log 2>&1 || exit $?
done
echo DONE
