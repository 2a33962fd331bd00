#!/bin/bash
# Build an alternate kernel library ab_libs/libghostm_hip_<tag>.so from the
# current sources with extra compile flags for device.hip (e.g. -DNAME=0), for
# same-box A/B runs (tools/ab.sh <tag>, or GHOSTM_LIB_PATH). Its GhostmBuildInfo
# says "A/B build <tag>"; ab_libs/ is git-ignored and deleted before suite runs
# (only ghostm_amd/lib's two product libraries ship with the tests).
#   tools/altlib.sh <tag> <flags...>
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; shift
B=$R/build/alt_$TAG
mkdir -p "$B"
make -C "$R/ghostm_amd/csrc" -s
mkdir -p "$R/ab_libs"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-result "$@" \
  "-DGHOSTM_ALT_TAG=\"$TAG\"" \
  -c "$R/ghostm_amd/csrc/device.hip" -o "$B/device.o"
N=$R/build/native
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$R/ab_libs/libghostm_hip_$TAG.so" \
  $N/formats.o $N/scoring.o $N/aligner.o $N/capi.o $N/formatter.o $N/synth.o $N/karlin_params.o $N/build_hash.o \
  "$B/device.o" $N/index.o $N/qformat.o -lpthread
echo "built ab_libs/libghostm_hip_$TAG.so"
