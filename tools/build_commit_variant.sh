#!/bin/bash
# Build the HIP library of a git commit into build/variants/<name>.so (A/B baselines for gpu_variants.sh).
# usage: tools/build_commit_variant.sh <commit> <name> [extra hipcc defines]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
c=$1; n=$2; shift 2
d=$(mktemp -d)
git -C "$R" archive "$c" dirt_amd/csrc include Makefile | tar -x -C "$d"
mkdir -p "$R/build/variants"
make -s -C "$d" variant NAME="$n" DEFS="$*" >/dev/null
cp "$d/build/variants/$n.so" "$R/build/variants/$n.so"
rm -rf "$d"
echo "built build/variants/$n.so from $(git -C "$R" rev-parse --short "$c")"
