#!/usr/bin/env bash
# Kernel-time sweep over env-selected variants: one rocprofv3 --kernel-trace --stats run of a short
# bench per variant.  usage: tools/variants.sh <tag> "<ENV=.. ENV=..>" ...   ("-" = defaults)
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
  env "${envs[@]}" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/v$n" -o run -- \
      python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --legs= --steps ${STEPS:-50} ${BENCH_EXTRA:-} > "$out/v$n.log" 2>&1
  rc=$?
  echo "=== variant $n [$v] rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$out/v$n.log"; exit $rc; }
  grep -h '^{' "$out/v$n.log" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('value %.3g  ms/step %.4f  frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['frac']))"
  f=$(find "$out/v$n" -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if int(r["Calls"]) >= 40:
        print("   %-60s calls %5s avg %8.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
