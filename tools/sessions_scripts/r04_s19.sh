#!/usr/bin/env bash
# round-4 session 19: clamped pick-up (ACSIM_BIN_POL bit 1024) parity, then A/B against the default
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_s19
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_binned.py tests/test_gpu_fullsize.py \
  -k "clamped or cache_policy or split or test_cfg4_full_size_bit_exact or packed" > gpurun_out/r04_s19/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r04_s19/tests.log; exit 1; }
tail -3 gpurun_out/r04_s19/tests.log
timeout -k 10 300 python -u tools/env_ab.py cfg4 200 4 "-;ACSIM_BIN_POL=1124" > gpurun_out/r04_s19/ab.jsonl 2>&1 || { echo ab failed; tail gpurun_out/r04_s19/ab.jsonl; exit 1; }
cat gpurun_out/r04_s19/ab.jsonl
