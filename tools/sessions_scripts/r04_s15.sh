#!/usr/bin/env bash
# round-4 session 14: double-buffered phase B (ACSIM_BIN_DB) parity, then A/B against the default
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_s15
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_binned.py tests/test_gpu_fullsize.py \
  -k "pipelined or double_buffered or split2 or test_cfg4_full_size_bit_exact" > gpurun_out/r04_s15/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r04_s15/tests.log; exit 1; }
tail -3 gpurun_out/r04_s15/tests.log
timeout -k 10 300 python -u tools/env_ab.py cfg4 200 3 "-;ACSIM_BIN_PP=1;ACSIM_BIN_PP=2;ACSIM_BIN_DB=1" > gpurun_out/r04_s15/ab.jsonl 2>&1 || { echo ab failed; tail gpurun_out/r04_s15/ab.jsonl; exit 1; }
cat gpurun_out/r04_s15/ab.jsonl
