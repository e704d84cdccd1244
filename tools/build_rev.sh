#!/bin/bash
# Build libmkidgpu.so as it was at a git revision, for same-process A/B timing (tools/kbench.py):
#   bash tools/build_rev.sh NAME REV [-- extra hipcc flags]
# exports mkids_sdr_amd/csrc and include/ at REV into a scratch dir (git archive, no checkout of
# this tree) and builds build/variants/NAME.so (gitignored; it travels to the GPU box).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REV=$2; shift 2
EXTRA=""
if [ $# -gt 0 ] && [ "$1" = "--" ]; then shift; EXTRA="$*"; fi
TMP=$(mktemp -d /tmp/mkidrev.XXXXXX)
git -C "$ROOT" archive "$REV" mkids_sdr_amd/csrc include | tar -x -C "$TMP"
mkdir -p "$ROOT/build/variants"
make -s -j8 -C "$TMP/mkids_sdr_amd/csrc" OUT="$ROOT/build/variants/$NAME.so" OBJDIR="$TMP/obj" EXTRA="$EXTRA" 2>&1 \
    | grep -v load-store-opt || true
rm -rf "$TMP"
ls -la "$ROOT/build/variants/$NAME.so"
