#!/usr/bin/env bash
# round 6: fp32 phase B on 128-receiver blocks (one pass, 8 workgroups per CU by LDS) against the
# default 256, after the phase-A change (tools/env_ab.py, alternating inside one build)
O=gpurun_out/r06_s14
mkdir -p $O
tools/gpu_session.sh r06_s14 \
  "300|python3 -u tools/env_ab.py cfg4_f32 100 6 '-;ACSIM_BIN_SB=128' > $O/sb_f32.jsonl"
