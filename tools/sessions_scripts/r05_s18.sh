#!/usr/bin/env bash
# round 5: Green's 16-wire network + merged 33-entry selection network (200 compare-exchanges for
# cfg4's window instead of 218) — GPU suite, same-box A/B against the round-4 network build
# (alternating processes: the library is chosen at import), and the round-time probe
O=gpurun_out/r05_s18
mkdir -p $O
V=tools/bin/batchernet/libacsim.so
AB4="for i in 1 2 3 4; do python3 tools/env_ab.py cfg4 200 1 - >> $O/ab_cfg4_new.jsonl && ACSIM_LIB=$V python3 tools/env_ab.py cfg4 200 1 - >> $O/ab_cfg4_old.jsonl || exit 1; done"
AB5="for i in 1 2; do python3 tools/env_ab.py cfg5 20 1 - >> $O/ab_cfg5_new.jsonl && ACSIM_LIB=$V python3 tools/env_ab.py cfg5 20 1 - >> $O/ab_cfg5_old.jsonl || exit 1; done"
tools/gpu_session.sh r05_s18 \
  "700|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu" \
  "400|$AB4" \
  "300|$AB5" \
  "200|python3 tools/round_phase_probe.py 5 20 > $O/phase_probe.jsonl" \
  "300|python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver1.json && ACSIM_LIB=$V python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver_old.json"
