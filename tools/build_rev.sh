#!/bin/bash
# Build libfasst_hip.so from the sources of a git revision into build/ab/NAME.so
# (same-box A/B baselines for tools/gpu_lib_ab.sh).  Usage: tools/build_rev.sh REV NAME
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
rev=$1; name=$2
tmp=$(mktemp -d /tmp/fasst_rev.XXXX)
git -C "$R" archive "$rev" pyfasst_amd/csrc include | tar -x -C "$tmp"
make -s -C "$tmp/pyfasst_amd/csrc" -j8 >/dev/null
mkdir -p "$R/build/ab"
cp "$tmp/pyfasst_amd/libfasst_hip.so" "$R/build/ab/$name.so"
rm -rf "$tmp"
echo "built build/ab/$name.so from $rev"
