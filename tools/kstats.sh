#!/usr/bin/env bash
# rocprofv3 kernel statistics of tools/bench_configs.py for the given presets.
# usage: tools/kstats.sh <tag> <preset>...
set -u
tag="$1"; shift
out="$GRAFT_REPO_ROOT/gpurun_out/$tag"
mkdir -p "$out"
cd /tmp; export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" "$@" > "$out/run.log" 2>&1
rc=$?
echo "rc=$rc"
f=$(find "$out" -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if float(r["TotalDurationNs"]) > 1e6:
        print("%-70s calls %6s avg %10.2f us  total %8.2f ms" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
exit $rc
