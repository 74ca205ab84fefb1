#!/usr/bin/env bash
# round 5: asm saddr LDS-DMA in phase B (ACSIM_BIN_POL bit 8192) — targeted tests, A/B, bench lines
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05_s12
mkdir -p $O
tools/gpu_session.sh r05_s12 \
  "400|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_binned.py tests/test_gpu_fullsize.py -k 'clamped or golden or eps_publication or cache_policy'" \
  "300|python3 tools/env_ab.py cfg4 200 4 '-;ACSIM_BIN_POL=13412;ACSIM_BIN_POL=1124' > $O/ab_cfg4.jsonl" \
  "300|python3 tools/env_ab.py cfg4_f32 200 2 '-;ACSIM_BIN_POL=13412' > $O/ab_cfg4_f32.jsonl"
