#!/bin/bash
# Build the working tree's library from a patched copy of csrc/ (a Python script edits the copy's
# tsdf_device.h in place) into abtest/lib<name>.so, for A/B runs (TSDF_HIP_LIB selects it).
#   tools/build_patched.sh <name> <patch.py | -> ["<extra hipcc flags>"]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/abpatch.XXXX)
mkdir -p "$W/pkg" "$W/include"
cp -r "$R/union-thesis-slam_amd/csrc" "$R/union-thesis-slam_amd/Makefile" "$W/pkg/"
cp "$R/include/"*.h "$W/include/"
[ "$2" != "-" ] && python3 "$2" "$W/pkg/csrc/tsdf_device.h"
make -s -j8 -C "$W/pkg" EXTRA="$3" >/dev/null
mkdir -p "$R/abtest"
cp "$W/pkg/tsdf_amd/lib/libtsdf_hip.so" "$R/abtest/lib$1.so"
rm -rf "$W"
echo "abtest/lib$1.so built (patch $2, flags '$3')"
