#!/usr/bin/env bash
# round 4: confirmation bench line with the keyed traffic / VALU / cfg5 traffic objects, and the
# rocprofv3 kernel statistics of the same command.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04_conf
tools/gpu_session.sh r04_conf \
  "300|python3 bench.py > $R/gpurun_out/r04_conf/bench.json" \
  "300|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04_conf/stats -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/r04_conf/bench_prof.json"
