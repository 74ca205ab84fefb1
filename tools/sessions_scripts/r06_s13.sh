#!/usr/bin/env bash
# round 6: re-sweep of phase-B passes and the fp32 stage-store flavour on the current sources
# (tools/env_ab.py, alternating inside one build)
O=gpurun_out/r06_s13
mkdir -p $O
tools/gpu_session.sh r06_s13 \
  "300|python3 -u tools/env_ab.py cfg4 100 4 '-;ACSIM_BIN_SPLIT=3;ACSIM_BIN_SPLIT=4' > $O/split_f64.jsonl" \
  "300|python3 -u tools/env_ab.py cfg4_f32 100 4 '-;ACSIM_BIN_SPLIT=2;ACSIM_BIN_POL=29728;ACSIM_BIN_POL=29730' > $O/f32_knobs.jsonl"
