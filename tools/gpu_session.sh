#!/usr/bin/env bash
# Run a sequence of GPU steps on the gpurun box, each under its own time limit.
# Usage: tools/gpu_session.sh <tag> <step>...   where each step is "SECONDS|command".
# Test failures (exit 1) do not stop the session; timeouts, aborts and crashes do
# (exit 124/134/137/139 or >128): nothing more touches the GPU after those.
set -u
tag="$1"; shift
out="gpurun_out/$tag"
mkdir -p "$out"
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n+1))
  secs="${step%%|*}"
  cmd="${step#*|}"
  echo "=== step $n (${secs}s): $cmd" | tee -a "$out/session.log"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/step$n.log" 2>&1
  rc=$?
  echo "=== step $n rc=$rc after $(( $(date +%s) - start ))s" | tee -a "$out/session.log"
  tail -n 25 "$out/step$n.log"
  if [ $rc -ge 124 ]; then
    echo "=== fatal rc=$rc: stopping the session" | tee -a "$out/session.log"
    exit $rc
  fi
done
exit 0
