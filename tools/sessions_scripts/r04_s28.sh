#!/usr/bin/env bash
# round-4 session 28: packed phase-M positions (ACSIM_BIN_PACK bit 3) parity, then A/B on cfg5
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_s28
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_binned.py tests/test_gpu_fullsize.py tests/test_gpu_f32.py \
  -k "packed or cfg5" > gpurun_out/r04_s28/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r04_s28/tests.log; exit 1; }
tail -3 gpurun_out/r04_s28/tests.log
timeout -k 10 400 python -u tools/env_ab.py cfg5 20 2 "-;ACSIM_BIN_MIMG=14336;ACSIM_BIN_PACK=9,ACSIM_BIN_MIMG=14336" > gpurun_out/r04_s28/ab_cfg5.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u tools/env_ab.py cfg5_f32 20 2 "-;ACSIM_BIN_PACK=9,ACSIM_BIN_MIMG=14336" > gpurun_out/r04_s28/ab_cfg5f32.jsonl 2>&1 || exit 1
echo done
