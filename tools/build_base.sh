#!/bin/bash
# A/B baseline: build the library of an earlier commit (a git worktree at
# /tmp/wt_base, default HEAD) as _lib/libtropical_hip_base.so, stamped with
# the CURRENT tree's build id so the loader accepts it under
# TNP_LIB=libtropical_hip_base.so (experiments only).
#   tools/build_base.sh [commit]
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
rev=${1:-HEAD}
[ -d /tmp/wt_base ] || git -C "$root" worktree add -f /tmp/wt_base "$rev" >/dev/null
git -C /tmp/wt_base checkout -q --detach "$(git -C "$root" rev-parse "$rev")"
id=$(sh "$root/tropical-nerf.pytorch_amd/csrc/build_id.sh")
make -C /tmp/wt_base/tropical-nerf.pytorch_amd/csrc -j8 BUILD_ID="$id" \
  OUT="$root/tropical-nerf.pytorch_amd/tropical/_lib/libtropical_hip_base.so" > /tmp/wt_base_build.log 2>&1
echo "base $(git -C /tmp/wt_base rev-parse --short HEAD) as libtropical_hip_base.so (id $id)"
