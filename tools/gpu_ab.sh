# Library A/B: for each "name=path" in $VARIANTS (path relative to the repo; "default" = in-tree build),
# per-launch probe of kernel class $PROBE (default 1 = GEMMs) and a short headline bench.
# A path may carry environment settings after commas: "name=default,KDLAE_X=1,KDLAE_Y=2".
# Optional $CHECK=1 first runs the T16-relevant GPU parity tests against every variant.
set -o pipefail
mkdir -p gpurun_out/ab
for nv in ${VARIANTS:-default=default}; do
  n=${nv%%=*}; v=${nv#*=}
  IFS=, read -r v envs <<< "$v"
  for e in ${envs//,/ }; do export "$e"; done
  if [ "$v" = default ]; then unset KDLAE_LIB; else export KDLAE_LIB=$GRAFT_REPO_ROOT/$v; fi
  if [ "${CHECK:-0}" = 1 ]; then
    timeout -k 10 400 python -u -m pytest tests/test_kdlae_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/gputest_$n.log 2>&1 || { tail -20 gpurun_out/ab/gputest_$n.log; exit 1; }
    echo "$n: $(tail -1 gpurun_out/ab/gputest_$n.log)"
  fi
  for c in ${PROBE:-1}; do
    KDLAE_PROBE_DUMP=gpurun_out/ab/probe_c${c}_$n.csv timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --probe $c --no-cpu-baseline --no-bs1 --no-secondary > gpurun_out/ab/probe_c${c}_$n.json 2> gpurun_out/ab/probe_c${c}_$n.err || exit $?
  done
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --probe 0 --no-cpu-baseline --no-bs1 --no-secondary > gpurun_out/ab/bench_$n.json 2> gpurun_out/ab/bench_$n.err || exit $?
  echo "$n: $(head -c 150 gpurun_out/ab/bench_$n.json)"
  for e in ${envs//,/ }; do unset "${e%%=*}"; done
done
