#!/bin/bash
# Build the working tree's libdronerl.so with extra kernel defines into
# scripts/micro/build/lib_$1.so (same-box A/B of kernel variants;
# DRONERL_LIB=... selects it).  Runs here (CPU).
#   bash scripts/micro/build_variant.sh nohbm "-DFL_NO_H"
set -e
tag=$1; flags=$2
root=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p "$root/scripts/micro/build"
make -s -C "$root/drone_rl_amd/csrc" -j8 OBJDIR="build_$tag" KFLAGS="$flags" \
     OUT="$root/scripts/micro/build/lib_$tag.so"
rm -rf "$root/drone_rl_amd/csrc/build_$tag"
echo "built scripts/micro/build/lib_$tag.so ($flags)"
