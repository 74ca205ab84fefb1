#!/usr/bin/env bash
# round 6: the default bench line and the driver's shape on the committed tree after the cfg5 leg's
# exit-code change (bench.py only; the kernels are unchanged)
tools/gpu_session.sh r06_s10 \
  "300|python3 -u bench.py > gpurun_out/r06_s10/bench_default.json" \
  "200|python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r06_s10/bench_driver.json"
