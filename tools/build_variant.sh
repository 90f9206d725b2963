#!/bin/bash
# Build librtzig.so from a git revision into ab/<name>.so (for in-process A/B, tools/ab_libs.py).
#   tools/build_variant.sh <rev|WORKTREE> <name>
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; NAME=$2
mkdir -p "$ROOT/ab"
if [ "$REV" = "WORKTREE" ]; then
  make -s -C "$ROOT/raytracing-with-zig_amd/csrc" >/dev/null
  cp "$ROOT/raytracing-with-zig_amd/librtzig.so" "$ROOT/ab/$NAME.so"
else
  WT=/tmp/rtwt_$NAME
  rm -rf "$WT"; git -C "$ROOT" worktree prune
  git -C "$ROOT" worktree add -f "$WT" "$REV" >/dev/null 2>&1
  make -s -C "$WT/raytracing-with-zig_amd/csrc" >/dev/null
  cp "$WT/raytracing-with-zig_amd/librtzig.so" "$ROOT/ab/$NAME.so"
  git -C "$ROOT" worktree remove --force "$WT"
fi
echo "ab/$NAME.so"
