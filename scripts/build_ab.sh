#!/bin/bash
# Build a library variant for side-by-side timing (scripts/ab_time.sh):
#   build_ab.sh NAME [REV]   -> ablibs/NAME/libpm.so from the csrc tree at git
#                              revision REV (default: the working tree)
# Extra hipcc flags via AB_HIPFLAGS (e.g. -DSOME_SWITCH; the kernels and the
# flattener both see them).
set -e
cd "$(dirname "$0")/.."
NAME=$1; REV=${2:-}
D=ablibs/$NAME; rm -rf "$D"; mkdir -p "$D/csrc" "$D/include"
if [ -n "$REV" ]; then
  mkdir -p "$D/tmp"; git archive "$REV" patternmatching_amd/csrc include | tar -x -C "$D/tmp"
  cp -r "$D/tmp/patternmatching_amd/csrc/." "$D/csrc/"; cp -r "$D/tmp/include/." "$D/include/"; rm -rf "$D/tmp"
else
  cp -r patternmatching_amd/csrc/. "$D/csrc/"; cp -r include/. "$D/include/"
fi
rm -rf "$D/csrc/build"
make -s -j8 -C "$D/csrc" ROOT="$(pwd)/$D" HIPFLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -I$(pwd)/$D/include -I$(pwd)/$D/csrc ${AB_HIPFLAGS:-}" FLATFLAGS="${AB_HIPFLAGS:-}" "$(pwd)/$D/libpm.so"
ls -la "$D/libpm.so"
