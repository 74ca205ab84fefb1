#!/usr/bin/env bash
# round 5: asm run copies in phase M and the one-pass phase B (ACSIM_BIN_POL bit 16384, opt-in) —
# bit-exactness cases, A/B on cfg5 (two-level) and cfg4 fp32 (one-pass phase B)
O=gpurun_out/r05_s16
mkdir -p $O
tools/gpu_session.sh r05_s16 \
  "400|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_binned.py -k 'asm_run_copies or clamped'" \
  "400|python3 tools/env_ab.py cfg5 20 3 '-;ACSIM_BIN_POL=29862' > $O/ab_cfg5.jsonl" \
  "300|python3 tools/env_ab.py cfg4_f32 200 4 '-;ACSIM_BIN_POL=29796;ACSIM_BIN_POL=29797' > $O/ab_cfg4_f32.jsonl"
