# Round 3: the full GPU suite as the driver runs it (no profiler), then smoke()
set -o pipefail
O=gpurun_out/${1:-suite}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rP --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
