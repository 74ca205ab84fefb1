#!/usr/bin/env bash
# round 5: new phase-B switches (tests + A/B), cfg5 phase-A segmentation sweep, cfg5 workgroup
# timestamps (phases A, M, B), cfg3 split-factor re-measurement
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05_s8
mkdir -p $O
tools/gpu_session.sh r05_s8 \
  "400|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_binned.py tests/test_gpu_fullsize.py -k 'clamped or golden or eps_publication or cache_policy'" \
  "300|python3 tools/env_ab.py cfg4 200 3 '-;ACSIM_BIN_POL=3172;ACSIM_BIN_POL=5220;ACSIM_BIN_POL=7268' > $O/ab_cfg4.jsonl" \
  "300|python3 tools/env_ab.py cfg5 10 1 '-;ACSIM_BIN_AWG=4096;ACSIM_BIN_AWG=8192;ACSIM_BIN_AWG=12288;ACSIM_BIN_AWG=16384;ACSIM_BIN_AWG=32768' > $O/awg_cfg5.jsonl" \
  "200|ACSIM_BIN_TS=$R/$O/ts_cfg5.csv python3 tools/env_ab.py cfg5 4 1 -" \
  "200|python3 tools/cfg3_shard_probe.py --reps 3 --no-events > $O/split2.jsonl && ACSIM_BATCH_SPLIT=4 python3 tools/cfg3_shard_probe.py --reps 3 --no-events > $O/split4.jsonl && ACSIM_BATCH_SPLIT=1 python3 tools/cfg3_shard_probe.py --reps 3 --no-events > $O/split1.jsonl"
