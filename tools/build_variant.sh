#!/bin/bash
# Build libfasst_hip.so from the WORKING TREE with extra compile flags into
# build/ab/NAME.so (same-box A/B of a -D switch).  Usage: tools/build_variant.sh NAME -DFOO=1 ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
tmp=$(mktemp -d /tmp/fasst_var.XXXX)
mkdir -p "$tmp/pyfasst_amd"
cp -r "$R/include" "$tmp/"
cp -r "$R/pyfasst_amd/csrc" "$tmp/pyfasst_amd/"
rm -f "$tmp"/pyfasst_amd/csrc/*.o
make -s -C "$tmp/pyfasst_amd/csrc" -j8 CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=true -Wall -Wno-unused-result -Wno-unused-value $*" >/dev/null
mkdir -p "$R/build/ab"
cp "$tmp/pyfasst_amd/libfasst_hip.so" "$R/build/ab/$name.so"
rm -rf "$tmp"
echo "built build/ab/$name.so with $*"
