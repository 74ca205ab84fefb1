#!/usr/bin/env bash
# round 5: EPS calls take their done count (and acs_round its states) through the host-mapped
# copy; acs_run's EPS end rides on the run summary — GPU suite, smoke, EPS presets' run() times
O=gpurun_out/r05_s28
mkdir -p $O
tools/gpu_session.sh r05_s28 \
  "700|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu" \
  "200|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|for i in 1 2 3; do python3 tools/bench_configs.py cfg4_eps cfg4_byz cfg4_fixed14 cfg1 cfg2 >> $O/configs_eps.jsonl || exit 1; done"
