#!/usr/bin/env bash
# round 6: fp32 phase-A workgroups per launch, per-kernel: rocprofv3 kernel traces of cfg4_f32 at
# 256 (the default) and 512 phase-A workgroups, alternating, plus a longer env A/B
O=gpurun_out/r06_s12
mkdir -p $O
tools/gpu_session.sh r06_s12 \
  "200|cd /tmp && rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/a256 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4_f32" \
  "200|cd /tmp && ACSIM_BIN_AWG=512 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/a512 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4_f32" \
  "200|cd /tmp && rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/b256 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4_f32" \
  "200|cd /tmp && ACSIM_BIN_AWG=512 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/b512 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4_f32" \
  "300|python3 -u tools/env_ab.py cfg4_f32 100 8 '-;ACSIM_BIN_AWG=512;ACSIM_BIN_AWG=384;ACSIM_BIN_AWG=768' > $O/awg_f32.jsonl" \
  "300|python3 -u tools/env_ab.py cfg5_f32 10 3 '-;ACSIM_BIN_AWG=8192' > $O/awg_cfg5_f32.jsonl"
