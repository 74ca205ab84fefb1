#!/usr/bin/env bash
# Build a variant libacsim.so under tools/bin/<name>/ (git-ignored; it travels to the GPU box) with
# extra compile flags for the named translation units; every other unit reuses csrc/build/*.o.
# Load it with ACSIM_LIB=tools/bin/<name>/libacsim.so (acsim/_abi.py).
# usage: tools/build_variant.sh <name> "<XFLAGS>" [unit.hip ...]   (default unit: round_binned.hip)
# A -D macro that a header (*.hpp) reads reaches every unit including that header, so such a flag
# rebuilds EVERY unit: a library mixing objects built with and without it would disagree on the
# header's constants (a 128-receiver phase B built into round_binned.hip alone, while
# api.hip still sized the block partials for 256).
set -eu
name="$1"; flags="$2"; shift 2
units="${*:-round_binned.hip}"
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C="$ROOT/approximate-consensus-simulation_amd/csrc"
out="$ROOT/tools/bin/$name"
for m in $(printf '%s\n' $flags | sed -n 's/^-D\([A-Za-z_][A-Za-z0-9_]*\).*/\1/p'); do
  if grep -qw "$m" "$C"/*.hpp "$ROOT"/include/*.h 2>/dev/null; then
    echo "build_variant: $m is read by a header: rebuilding every unit" >&2
    units=$(cd "$C" && ls *.hip)
    break
  fi
done
mkdir -p "$out/obj"
make -s -C "$C" >/dev/null            # the default objects are current
cp -p "$C"/build/*.o "$out/obj/"
for u in $units; do rm -f "$out/obj/${u%.hip}.o"; done
make -s -C "$C" OBJDIR="$out/obj" OUTDIR="$out" XFLAGS="$flags"
echo "$out/libacsim.so"
