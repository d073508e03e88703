#!/bin/bash
# Build libjaadgpu.so of git revision REV into .tmp/exp/lib_NAME.so (a same-call A/B baseline):
#   bash scripts/build_rev_variant.sh REV NAME
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=/tmp/jaad_wt_$2
rm -rf "$WT"; git -C "$ROOT" worktree prune
git -C "$ROOT" worktree add -f --detach "$WT" "$1" > /dev/null
mkdir -p "$ROOT/.tmp/exp"
(cd "$WT" && python3 -c "from jaadec_amd import build as B; B.build_gpu(out=__import__('pathlib').Path('$ROOT/.tmp/exp/lib_$2.so'), force=True)" > /tmp/build_rev_$2.log 2>&1)
git -C "$ROOT" worktree remove --force "$WT"
echo "built .tmp/exp/lib_$2.so from $1"
