#!/bin/bash
# Build a libmkidgpu.so variant for same-process A/B timing (tools/kbench.py):
#   bash tools/build_variant.sh NAME [REV:FILE ...] [-- extra hipcc flags]
# copies mkids_sdr_amd/csrc to a scratch dir, replaces each FILE (relative to csrc) by its content at
# git revision REV, and builds build/variants/NAME.so (gitignored; it travels to the GPU box).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
TMP=$(mktemp -d /tmp/mkidvar.XXXXXX)
mkdir -p "$TMP/pkg" && cp -r "$ROOT/mkids_sdr_amd/csrc" "$TMP/pkg/csrc"
mkdir -p "$TMP/include" && cp "$ROOT/include/"*.h "$TMP/include/"
EXTRA=""
while [ $# -gt 0 ]; do
    if [ "$1" = "--" ]; then shift; EXTRA="$*"; break; fi
    REV=${1%%:*}; F=${1#*:}
    git -C "$ROOT" show "$REV:mkids_sdr_amd/csrc/$F" > "$TMP/pkg/csrc/$F"
    shift
done
mkdir -p "$ROOT/build/variants"
make -s -C "$TMP/pkg/csrc" OUT="$ROOT/build/variants/$NAME.so" OBJDIR="$TMP/obj" EXTRA="$EXTRA" 2>&1 | grep -v load-store-opt || true
rm -rf "$TMP"
ls -la "$ROOT/build/variants/$NAME.so"
