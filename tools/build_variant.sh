#!/bin/bash
# Build a libkdlae.so variant for same-box A/Bs (tools/gpu.sh ab / VARIANTS=name=build_ab/<name>/libkdlae.so):
#   tools/build_variant.sh <name> <git-rev|-> [file=path-to-replacement ...] [-- extra hipcc flags]
# (tuning constants are constexpr in the sources since r06: change one through a file replacement)
# Copies csrc (from <git-rev>, or the working tree with -) and include/ to build_ab/<name>/, replaces the
# listed files, and builds build_ab/<name>/libkdlae.so.  build_ab/ is git-ignored.
set -e
name=$1; rev=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
D=$R/build_ab/$name
rm -rf "$D"; mkdir -p "$D/pkg/csrc" "$D/include"
if [ "$rev" = - ]; then
  cp "$R"/rethink_acoustic_image_enhancement_amd/csrc/*.{hip,cpp,h} "$R"/rethink_acoustic_image_enhancement_amd/csrc/Makefile "$D/pkg/csrc/"
  cp "$R"/include/kdlae.h "$D/include/"
else
  for f in $(git -C "$R" ls-tree --name-only "$rev" rethink_acoustic_image_enhancement_amd/csrc/); do
    git -C "$R" show "$rev:$f" > "$D/pkg/csrc/$(basename $f)"
  done
  git -C "$R" show "$rev:include/kdlae.h" > "$D/include/kdlae.h"
fi
extra=""
while [ $# -gt 0 ]; do
  case $1 in
    --) shift; extra="$*"; break ;;
    *=*) cp "${1#*=}" "$D/pkg/csrc/${1%%=*}" ;;
  esac
  shift
done
make -C "$D/pkg/csrc" -j8 OUT=../../libkdlae.so BUILD=build EXTRA="$extra" > "$D/build.log" 2>&1 || { tail -20 "$D/build.log"; exit 1; }
echo "$D/libkdlae.so"
