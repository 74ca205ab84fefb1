#!/usr/bin/env bash
# round 5: asm saddr LDS-DMA with the pad bits masked off the run start — GPU suite (with the
# bit-8192 cases), A/B against the default, bench lines
O=gpurun_out/r05_s15
mkdir -p $O
tools/gpu_session.sh r05_s15 \
  "700|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu" \
  "400|python3 tools/env_ab.py cfg4 200 4 '-;ACSIM_BIN_POL=13412' > $O/ab_cfg4.jsonl" \
  "300|python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver1.json && ACSIM_BIN_POL=13412 python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver_asm.json"
