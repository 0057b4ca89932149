#!/bin/bash
# Build libdronerl.so from the kernel sources of git revision $1 into
# scripts/micro/build/lib_$2.so (for same-box A/B runs against the working
# tree; DRONERL_LIB=... selects it).  Runs here (CPU), hipcc cross-compiles.
set -e
rev=$1; tag=$2
root=$(cd "$(dirname "$0")/../.." && pwd)
tmp=$(mktemp -d)
mkdir -p "$tmp/drone_rl_amd/csrc" "$tmp/include" "$root/scripts/micro/build"
git -C "$root" archive "$rev" drone_rl_amd/csrc include | tar -x -C "$tmp"
make -s -C "$tmp/drone_rl_amd/csrc" -j8 OUT="$root/scripts/micro/build/lib_$tag.so"
rm -rf "$tmp"
echo "built scripts/micro/build/lib_$tag.so from $rev"
