#!/bin/bash
# Build the working tree's library with extra compiler flags into abtest/lib<name>.so (A/B runs
# select it with TSDF_HIP_LIB).   tools/build_variant.sh <name> "<extra hipcc flags>"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/abvar.XXXX)
mkdir -p "$W/pkg" "$W/include"
cp -r "$R/union-thesis-slam_amd/csrc" "$R/union-thesis-slam_amd/Makefile" "$W/pkg/"
cp "$R/include/"*.h "$W/include/"
make -s -C "$W/pkg" EXTRA="$2" >/dev/null
mkdir -p "$R/abtest"
cp "$W/pkg/tsdf_amd/lib/libtsdf_hip.so" "$R/abtest/lib$1.so"
rm -rf "$W"
echo "abtest/lib$1.so built with: $2"
