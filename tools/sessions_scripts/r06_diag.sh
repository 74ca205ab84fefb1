#!/usr/bin/env bash
# round 6: byte / LDS diagnostics against the default build, kernel stats
# of 100 FIXED cfg4 rounds per library: diagb4 = phase B without its invpos stream, diaga1 = phase A
# with bank-conflict-free LDS reads (both wrong values by design; tools/build_variant.sh)
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r06_diag
mkdir -p $out
cd /tmp; export TMPDIR=/tmp
for v in default diagb4 diaga1 default2 diagb4_2 diaga1_2; do
  b=${v%_2}; b=${b%2}
  lib=$R/approximate-consensus-simulation_amd/acsim/_lib/libacsim.so
  [ $b != default ] && lib=$R/tools/bin/$b/libacsim.so
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
