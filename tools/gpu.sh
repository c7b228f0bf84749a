# GPU-box recipes (run through gpurun from the repo root), one subcommand per call:
#   bash tools/gpu.sh <cmd> <outdir-under-gpurun_out> [args]
# Every GPU step has its own time limit and the first failure ends the script (no retries).
#   suite     kernel-variant tests, then the rest of the GPU suite (one pytest process each)
#   tests     pytest on the given test files / node ids (args)
#   smoke     __graft_entry__.smoke()
#   bench     bench.py with the given args (default: the driver's default run)
#   prof      rocprofv3 --kernel-trace --stats of the T16 bench and of the training bench
#   profb     rocprofv3 --kernel-trace --stats of one bench.py run with the given args
#   probe     a tools/ probe script with args, then the same under rocprofv3 --kernel-trace --stats
#   pmc_lds   one PMC pass of wave-state + LDS counters over one T16 step
#   split     tools/stream_split_probe.py (two half-batches on two streams vs one)
#   pmc       PMC passes over one T16 step: FETCH_SIZE, WRITE_SIZE, busy counters (one group per run)
#   ab        library A/B: for each "name=path[,ENV=V...]" in $VARIANTS ("default" = in-tree build), the
#             per-launch probe of class $PROBE (default 1) and a short T16 bench; CHECK=1 runs
#             tests/test_kdlae_gpu.py against each variant first
#   train_ab  like ab for the training step: launch trace (tools/train_trace.py) + training bench
#   trains_ab the KDLAE-S training bench for each variant
#   taps      tools/config1_taps.py gpu leg for each "name=path" in $VARIANTS
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cmd=$1
O=$R/gpurun_out/${2:-$cmd}
shift 2 2>/dev/null || shift $#
mkdir -p "$O"
cd "$R"
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"

use_variant() {  # name=path[,ENV=V...] -> exports; prints the name
  local nv=$1 n v envs
  unset KDLAE_DEBUG  # a previous variant's environment must not leak into this one
  n=${nv%%=*}; v=${nv#*=}
  IFS=, read -r v envs <<< "$v"
  for e in ${envs//,/ }; do export "$e"; done
  if [ "$v" = default ]; then unset KDLAE_LIB; else export KDLAE_LIB=$R/$v; fi
  VNAME=$n
}

case $cmd in
suite)
  timeout -k 10 400 $PYT tests/test_kernel_variants_infer_gpu.py tests/test_kernel_variants_gpu.py > $O/variants.log 2>&1 || { tail -40 $O/variants.log; exit 1; }
  tail -2 $O/variants.log
  timeout -k 10 700 $PYT tests -m gpu -v --deselect tests/test_kernel_variants_infer_gpu.py --deselect tests/test_kernel_variants_gpu.py > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
  tail -2 $O/gputest.log
  ;;
tests)
  timeout -k 10 600 $PYT -v "$@" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
  ;;
smoke)
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
  cat $O/smoke.log
  ;;
bench)
  timeout -k 10 600 python -u bench.py "$@" > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
  head -c 600 $O/bench.json; echo
  ;;
prof)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-bs1 --no-secondary --no-train > $O/prof_bench.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_train -o run -- python3 $R/bench.py --workload train --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_train.log 2>&1 || exit $?
  ;;
profb)  # rocprofv3 kernel trace + stats of one bench.py invocation (args)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py "$@" > $O/prof_bench.log 2>&1 || exit $?
  tail -2 $O/prof_bench.log
  ;;
probe)  # a tools/ probe script (args: script [script args]), then the same under rocprofv3 --kernel-trace --stats
  timeout -k 10 300 python -u "$@" > $O/probe.txt 2> $O/probe.err || { tail -30 $O/probe.err; exit 1; }
  cat $O/probe.txt
  s=$R/$1; shift
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $s "$@" > $O/prof_probe.log 2>&1 || exit $?
  ;;
pmc_sec)  # FETCH_SIZE / WRITE_SIZE passes over one S8 and one A64 forward -> profiles-ready json
  cd /tmp && export TMPDIR=/tmp
  for w in s8 a64; do
    B="python3 $R/bench.py --workload $w --steps 1 --warmup 0 --no-cpu-baseline"
    timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${w}_fetch -o run -- $B > $O/${w}_fetch.log 2>&1 || exit $?
    timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${w}_write -o run -- $B > $O/${w}_write.log 2>&1 || exit $?
    python3 $R/tools/pmc_workload.py $(ls $O/${w}_fetch/*counter_collection.csv | head -1) \
      $(ls $O/${w}_write/*counter_collection.csv | head -1) $O/pmc_$w.json $w || exit $?
  done
  ;;
pmc)
  cd /tmp && export TMPDIR=/tmp
  B="python3 $R/bench.py --steps 1 --warmup 0 --probe 0 --no-cpu-baseline --no-bs1 --no-secondary --no-train"
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B > $O/pmc_fetch.log 2>&1 || exit $?
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B > $O/pmc_write.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_busy -o run -- $B > $O/pmc_busy.log 2>&1 || exit $?
  # per-class traffic of this build (lib_sha256 recorded), warm-up forward included: 2 forwards
  python3 $R/tools/pmc_summary.py $(ls $O/pmc_fetch/*counter_collection.csv | head -1) \
    $(ls $O/pmc_write/*counter_collection.csv | head -1) $O/pmc_traffic.json > $O/pmc_traffic.log 2>&1 || exit $?
  python3 $R/tools/pmc_busy.py $(ls $O/pmc_busy/*counter_collection.csv | head -1) $O/pmc_busy.json r06 > $O/pmc_busy_sum.log 2>&1 || exit $?
  ;;
pmc_lds)  # one T16 step: wave-state and LDS counters per kernel (one pass)
  cd /tmp && export TMPDIR=/tmp
  B="python3 $R/bench.py --steps 1 --warmup 0 --probe 0 --no-cpu-baseline --no-bs1 --no-secondary --no-train"
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $O/pmc_lds -o run -- $B > $O/pmc_lds.log 2>&1 || exit $?
  ;;
split)  # two half-batches on two streams vs one stream (tools/stream_split_probe.py)
  timeout -k 10 300 python -u tools/stream_split_probe.py ${STEPS:-5} > $O/split.json 2> $O/split.err || { tail -20 $O/split.err; exit 1; }
  cat $O/split.json
  ;;
ab)
  for nv in ${VARIANTS:-default=default}; do
    use_variant "$nv"; n=$VNAME
    if [ "${CHECK:-0}" = 1 ]; then
      timeout -k 10 400 $PYT tests/test_kdlae_gpu.py > $O/gputest_$n.log 2>&1 || { tail -20 $O/gputest_$n.log; exit 1; }
      echo "$n: $(tail -1 $O/gputest_$n.log)"
    fi
    for c in ${PROBE:-1}; do
      KDLAE_PROBE_DUMP=$O/probe_c${c}_$n.csv timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --probe $c --probe-steps 2 --no-cpu-baseline --no-bs1 --no-secondary > $O/probe_c${c}_$n.json 2> $O/probe_c${c}_$n.err || exit $?
    done
    timeout -k 10 300 python -u bench.py --steps ${STEPS:-5} --warmup 2 --probe 0 --no-cpu-baseline --no-bs1 --no-secondary > $O/bench_$n.json 2> $O/bench_$n.err || exit $?
    echo "$n: $(head -c 150 $O/bench_$n.json)"
  done
  ;;
train_ab)
  for nv in ${VARIANTS:-default=default}; do
    use_variant "$nv"; n=$VNAME
    timeout -k 10 300 python -u tools/train_trace.py $O/$n.csv > $O/$n.txt 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
    echo "$n: $(head -1 $O/$n.txt)"
    timeout -k 10 300 python -u bench.py --workload train --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
    echo "$n bench: $(head -c 200 $O/bench_$n.json)"
  done
  ;;
trains_ab)  # KDLAE-S training bench per variant
  for nv in ${VARIANTS:-default=default}; do
    use_variant "$nv"; n=$VNAME
    timeout -k 10 300 python -u bench.py --workload train_s --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_s_$n.json 2> $O/bench_s_$n.err || { tail -20 $O/bench_s_$n.err; exit 1; }
    echo "$n train_s bench: $(head -c 200 $O/bench_s_$n.json)"
  done
  ;;
taps)
  for nv in ${VARIANTS:-base=default}; do
    use_variant "$nv"
    timeout -k 10 300 python -u tools/config1_taps.py gpu --tag $VNAME --out $O > $O/taps_$VNAME.log 2>&1 || { tail -20 $O/taps_$VNAME.log; exit 1; }
    tail -1 $O/taps_$VNAME.log
  done
  ;;
*)
  echo "unknown subcommand $cmd"; exit 2 ;;
esac
