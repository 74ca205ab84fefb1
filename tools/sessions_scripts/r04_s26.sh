#!/usr/bin/env bash
# round-4 session 26: fp32 packed phase-A indices (ACSIM_BIN_PACK bit 2) parity, then A/B of fp32
# source-block size and packing on cfg4_f32 and cfg5_f32
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_s26
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_f32.py tests/test_gpu_fullsize.py \
  -k "packed or f32" > gpurun_out/r04_s26/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r04_s26/tests.log; exit 1; }
tail -3 gpurun_out/r04_s26/tests.log
timeout -k 10 300 python -u tools/env_ab.py cfg4_f32 200 3 "-;ACSIM_BIN_SA=16384;ACSIM_BIN_SA=16384,ACSIM_BIN_PACK=5" > gpurun_out/r04_s26/ab_cfg4f32.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u tools/env_ab.py cfg5_f32 20 2 "-;ACSIM_BIN_SA=16384;ACSIM_BIN_SA=16384,ACSIM_BIN_PACK=5" > gpurun_out/r04_s26/ab_cfg5f32.jsonl 2>&1 || exit 1
echo done
