#!/usr/bin/env bash
# round 4, session 13: every preset on this build and on the round-3 build (regression check).
R=$GRAFT_REPO_ROOT
O=$R/tools/sessions/0eb899f
P="cfg1 cfg2 cfg3 cfg3_g16 cfg4 cfg4_eps cfg4_byz cfg5 cfg4_f32 cfg3_f32 cfg5_f32 cfg4_byz_f32 csr_2e20 csr_2e20_hubs"
tools/gpu_session.sh r04_s13 \
  "600|python3 tools/bench_configs.py $P" \
  "600|cd $O && python3 tools/bench_configs.py $P"
