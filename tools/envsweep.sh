#!/usr/bin/env bash
# Headline bench line under several environment settings (one process each, 60 s limit each).
# usage: tools/envsweep.sh "ENV=.. ENV2=.." "ENV=.." ...   ("-" = defaults)
for e in "$@"; do
  [ "$e" = "-" ] && e=""
  out=$(env $e timeout -k 10 60 python bench.py --steps 50 --warmup 10 --legs "" --no-cpu-baseline 2>&1 | grep '^{')
  rc=$?
  python3 - "$e" "$out" <<'PY'
import json, sys
e, line = sys.argv[1], sys.argv[2]
try:
    d = json.loads(line)
    print(f"{e or 'default':40s} {d['value']/1e9:7.3f} G  ms {d['ms_per_step']*1e3:7.2f} us  launch {d['roofline']['avg_launch_us']:7.2f} us  frac {d['roofline']['frac']:.4f}  golden {d['parity']['golden_match']}")
except Exception as ex:
    print(e, "FAILED", ex, line[:200])
PY
  [ $rc -ge 124 ] && exit $rc
done
exit 0
