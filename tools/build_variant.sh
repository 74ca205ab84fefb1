#!/usr/bin/env bash
# Build a variant libacsim.so under tools/bin/<name>/ (git-ignored; it travels to the GPU box) with
# extra compile flags for the named translation units; every other unit reuses csrc/build/*.o.
# Load it with ACSIM_LIB=tools/bin/<name>/libacsim.so (acsim/_abi.py).
# usage: tools/build_variant.sh <name> "<XFLAGS>" [unit.hip ...]   (default unit: round_binned.hip)
set -eu
name="$1"; flags="$2"; shift 2
units="${*:-round_binned.hip}"
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C="$ROOT/approximate-consensus-simulation_amd/csrc"
out="$ROOT/tools/bin/$name"
mkdir -p "$out/obj"
make -s -C "$C" >/dev/null            # the default objects are current
cp -p "$C"/build/*.o "$out/obj/"
for u in $units; do rm -f "$out/obj/${u%.hip}.o"; done
make -s -C "$C" OBJDIR="$out/obj" OUTDIR="$out" XFLAGS="$flags"
echo "$out/libacsim.so"
