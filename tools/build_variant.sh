#!/bin/bash
# Build librtzig.so from a git revision into ab/<name>.so (for in-process A/B, tools/ab_libs.py).
#   tools/build_variant.sh <rev|WORKTREE> <name>
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; NAME=$2
mkdir -p "$ROOT/ab"
if [ "$REV" = "WORKTREE" ]; then
  # EXTRA: extra compiler flags for ablation builds (e.g. -DRTZIG_RUV_TRIPS=2), built out of tree
  if [ -n "$EXTRA" ]; then
    B=/tmp/rtab_$NAME; rm -rf "$B"; mkdir -p "$B"
    C="$ROOT/raytracing-with-zig_amd/csrc"
    F="-O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-function $EXTRA"
    /opt/rocm/bin/hipcc $F -x hip --offload-arch=gfx950 -fno-gpu-rdc -c "$C/rt_kernel.hip" -o "$B/k.o"
    /opt/rocm/bin/hipcc $F -x hip --offload-arch=gfx950 -fno-gpu-rdc -c "$C/rt_runtime.cpp" -o "$B/r.o"
    /opt/rocm/bin/hipcc $F -x c++ -c "$C/rt_host.cpp" -o "$B/h.o"
    /opt/rocm/bin/hipcc $F -x c++ -c "$C/rt_bvh.cpp" -o "$B/b.o"
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$ROOT/ab/$NAME.so" "$B"/*.o
    echo "ab/$NAME.so"; exit 0
  fi
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
