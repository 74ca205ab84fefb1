#!/usr/bin/env bash
# round 5: phase-B diagnostics (tools/build_variant.sh diagb1..3) against the default build, kernel stats
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r05_diagb
mkdir -p $out
cd /tmp; export TMPDIR=/tmp
for v in default diagb1 diagb2 diagb3 default; do
  lib=$R/approximate-consensus-simulation_amd/acsim/_lib/libacsim.so
  [ $v != default ] && lib=$R/tools/bin/$v/libacsim.so
  ACSIM_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$v -o run -- \
      python3 $R/tools/env_ab.py cfg4 100 1 - > $out/$v.log 2>&1 || exit $?
  f=$(find $out/$v -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if int(r["Calls"]) >= 50:
        print(sys.argv[2], "%-50s calls %5s avg %8.2f us" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
