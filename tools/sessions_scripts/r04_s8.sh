#!/usr/bin/env bash
# round 4, session 8: per-phase kernel time of the packed streams (phase A / phase B / both / none).
R=$GRAFT_REPO_ROOT
steps=()
for rep in 1 2; do for P in 0 1 2 3; do
  steps+=("200|cd /tmp && ACSIM_BIN_PACK=$P rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04_s8_p${P}_r$rep -o run -- python3 $R/tools/pol_ab.py cfg4 200 65536 1")
done; done
tools/gpu_session.sh r04_s8 "${steps[@]}" \
  "200|for i in 1 2; do for P in 0 1 2 3; do ACSIM_BIN_PACK=\$P python3 tools/pol_ab.py cfg4 200 65536 1; done; done"
