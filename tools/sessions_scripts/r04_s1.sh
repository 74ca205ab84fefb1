#!/usr/bin/env bash
# round 4, session 1: cfg5 current vs round-2 head (3258e05, built under tools/sessions/r02), A/B/A/B,
# then kernel stats of both, then a fresh headline bench line.
R=$GRAFT_REPO_ROOT
OLD=$R/tools/sessions/r02
tools/gpu_session.sh r04_s1 \
 "200|python3 tools/bench_configs.py cfg5 cfg5_f32" \
 "200|cd $OLD && python3 tools/bench_configs.py cfg5 cfg5_f32" \
 "200|python3 tools/bench_configs.py cfg5 cfg5_f32" \
 "200|cd $OLD && python3 tools/bench_configs.py cfg5 cfg5_f32" \
 "250|tools/kstats.sh r04_s1_kcur cfg5" \
 "250|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04_s1_kold -o run -- python3 $OLD/tools/bench_configs.py cfg5" \
 "200|python3 bench.py --legs f32,cfg3,cfg5 --no-cpu-baseline"
