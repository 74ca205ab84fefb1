#!/usr/bin/env bash
# tools/variants.sh with the bench in fp32 mode.  usage: tools/variants_f32.sh <tag> "<ENV=..>" ...
export BENCH_EXTRA="--dtype f32"
exec bash "$(dirname "$0")/variants.sh" "$@"
