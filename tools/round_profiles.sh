#!/usr/bin/env bash
# Round-end evidence: bench lines (fp64 headline, fp32 mode), rocprofv3 kernel stats of both bench
# commands, and the FETCH_SIZE / WRITE_SIZE passes for the traffic figure.  usage: tools/round_profiles.sh <tag>
set -u
tag="$1"
out="$GRAFT_REPO_ROOT/gpurun_out/$tag"
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
B="$GRAFT_REPO_ROOT/bench.py"
timeout -k 10 300 python3 "$B" > "$out/bench_f64.json" 2> "$out/bench_f64.err" || exit $?
timeout -k 10 300 python3 "$B" --dtype f32 > "$out/bench_f32.json" 2> "$out/bench_f32.err" || exit $?
for dt in f64 f32; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats_$dt" -o run -- \
      python3 "$B" --no-cpu-baseline --legs= --dtype $dt > "$out/stats_$dt.log" 2>&1 || exit $?
  for pass in "FETCH_SIZE" "WRITE_SIZE"; do
    timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$out/pmc_${dt}_$pass" -o run -- \
        python3 "$B" --no-cpu-baseline --legs= --dtype $dt --steps 30 > "$out/pmc_${dt}_$pass.log" 2>&1 || exit $?
  done
done
echo done
