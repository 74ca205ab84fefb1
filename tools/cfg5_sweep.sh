#!/usr/bin/env bash
# cfg5 kernel times per env-selected variant (rocprofv3 kernel stats of tools/bench_configs.py cfg5).
# usage: tools/cfg5_sweep.sh <tag> "<ENV=..>" ...   ("-" = defaults; CFG=cfg5_f32 for fp32)
set -u
tag="$1"; shift
out="$GRAFT_REPO_ROOT/gpurun_out/$tag"
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
n=0
for v in "$@"; do
  n=$((n+1))
  envs=()
  [ "$v" != "-" ] && read -r -a envs <<< "$v"
  env "${envs[@]}" timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/v$n" -o run -- \
      python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" ${CFG:-cfg5} > "$out/v$n.log" 2>&1
  rc=$?
  echo "=== variant $n [$v] rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$out/v$n.log"; exit $rc; }
  f=$(find "$out/v$n" -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if int(r["Calls"]) >= 20:
        print("   %-60s calls %5s avg %9.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
