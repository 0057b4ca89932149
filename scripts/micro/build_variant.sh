#!/bin/bash
# Build the working tree's libdronerl.so with extra kernel defines into
# scripts/micro/build/lib_$1.so (same-box A/B of kernel variants;
# DRONERL_LIB=... selects it).  Runs here (CPU).  An optional third argument
# names a patch (scripts/micro/patches/*.patch: `git diff` form, applied with
# -p1 at the repo root) applied to a scratch copy of the kernel sources
# first.  The diagnostic, wrong-result ablation switches (DR_ABLATE,
# DR_WS_ABL, FL_NO_H / FL_NO_D2, DR_LT_ABL, DR_HEAD_DIAG) live only in those
# patches, never in the product sources (verdict r05 item 3).
#   bash scripts/micro/build_variant.sh m16 "-DX6_MFMA16=1"
#   bash scripts/micro/build_variant.sh nohbm "-DFL_NO_H" scripts/micro/patches/x6_diag.patch
set -e
tag=$1; flags=$2; patchf=$3
root=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p "$root/scripts/micro/build"
src="$root"
if [ -n "$patchf" ]; then
    pabs=$(cd "$(dirname "$patchf")" && pwd)/$(basename "$patchf")
    src=$(mktemp -d)
    mkdir -p "$src/drone_rl_amd" "$src/include"
    cp -r "$root/drone_rl_amd/csrc" "$src/drone_rl_amd/"
    rm -rf "$src"/drone_rl_amd/csrc/build*
    cp "$root/include/dronerl.h" "$src/include/"
    patch -s -p1 -d "$src" < "$pabs"
fi
make -s -C "$src/drone_rl_amd/csrc" -j8 OBJDIR="build_$tag" KFLAGS="$flags" \
     OUT="$root/scripts/micro/build/lib_$tag.so"
rm -rf "$src/drone_rl_amd/csrc/build_$tag"
if [ "$src" != "$root" ]; then rm -rf "$src"; fi
echo "built scripts/micro/build/lib_$tag.so ($flags${patchf:+, $patchf})"
