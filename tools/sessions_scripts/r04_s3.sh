#!/usr/bin/env bash
# round 4, session 3: binned parity with the packed phase-A indices, stage-store policy A/B inside
# one build (cfg4, cfg5), packed vs u16 indices, cfg3 size sweep and a cfg3 shard timeline.
R=$GRAFT_REPO_ROOT
tools/gpu_session.sh r04_s3 \
  "400|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_binned.py tests/test_gpu_fullsize.py -k 'binned or cfg4 or cfg5 or policy or split or eps_pub' -m gpu" \
  "200|python3 tools/pol_ab.py cfg4 200 36,38,100 3" \
  "200|for i in 1 2 3; do ACSIM_BIN_PACK=0 python3 tools/pol_ab.py cfg4 200 36 1; ACSIM_BIN_PACK=1 python3 tools/pol_ab.py cfg4 200 36 1; done" \
  "400|python3 tools/pol_ab.py cfg5 30 36,38,164,166,292 2" \
  "200|python3 tools/cfg3_size_sweep.py --timing 1" \
  "200|python3 tools/cfg3_size_sweep.py --timing 0" \
  "200|cd /tmp && rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $R/gpurun_out/r04_s3_cfg3tl -o run -- python3 $R/tools/cfg3_size_sweep.py --timing 0 --sizes 12500,100000 --reps 3"
