#!/usr/bin/env bash
# round 6: phase-A workgroups per launch for the fp32 headline (x block 64 KiB: two workgroups fit a
# CU's LDS, so one can stage while the other streams) and the fp64 one (128 KiB: one per CU), A/B
# inside one build (tools/env_ab.py)
O=gpurun_out/r06_s11
mkdir -p $O
tools/gpu_session.sh r06_s11 \
  "300|python3 -u tools/env_ab.py cfg4_f32 100 4 '-;ACSIM_BIN_AWG=512;ACSIM_BIN_AWG=1024' > $O/awg_f32.jsonl" \
  "300|python3 -u tools/env_ab.py cfg4 100 4 '-;ACSIM_BIN_AWG=512' > $O/awg_f64.jsonl"
