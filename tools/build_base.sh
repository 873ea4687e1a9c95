#!/bin/bash
# Build libsad.so from a git revision (default HEAD) into abl/libsad_<tag>.so
# for same-box A/B runs (SAD_LIB=... python bench.py): bash tools/build_base.sh [rev] [tag]
set -e
REV=${1:-HEAD}; TAG=${2:-base}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$ROOT" archive "$REV" synthetic-audio-detection_amd/csrc include | tar -x -C "$T"
mkdir -p "$ROOT/abl"
make -C "$T/synthetic-audio-detection_amd/csrc" -j8 OUT="$ROOT/abl/libsad_$TAG.so" BUILD="$T/obj" >/dev/null
rm -rf "$T"
echo "$ROOT/abl/libsad_$TAG.so"
