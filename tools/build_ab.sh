#!/bin/bash
# Build the library of git revision $1 (default HEAD) into abtest/libB.so, for tools/gpu/run_ab.sh.
set -e
REV=${1:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/abwt.XXXX)
git -C "$R" worktree add -q --detach "$W" "$REV"
make -s -C "$W/union-thesis-slam_amd"
mkdir -p "$R/abtest"
cp "$W/union-thesis-slam_amd/tsdf_amd/lib/libtsdf_hip.so" "$R/abtest/libB.so"
git -C "$R" worktree remove --force "$W"
echo "abtest/libB.so <- $REV"
