#!/usr/bin/env bash
# round 6, final evidence part 3: complete default and fp32 bench lines with every counter summary
# keyed to these sources in the tree (the cfg3 VALU roofline included)
O=gpurun_out/r06_fin9
mkdir -p $O
tools/gpu_session.sh r06_fin9 \
  "300|python3 -u bench.py > $O/bench_default.json" \
  "300|python3 -u bench.py --dtype f32 > $O/bench_f32.json"
