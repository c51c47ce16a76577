#!/bin/bash
# Build commit $1's libraries into ab_base/ (for scripts/gpu_ab_libs.sh), from a temporary worktree.
set -e
C=${1:?commit}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/abbase.XXXXXX)
git -C "$ROOT" worktree add --detach "$T" "$C" > /dev/null
make -s -j 8 -C "$T/chiaroscuro-raytracer_amd" lib/libchiaro_hip.so lib/libchiaroscuro.so
mkdir -p "$ROOT/ab_base"
cp "$T/chiaroscuro-raytracer_amd/lib/"*.so "$ROOT/ab_base/"
git -C "$ROOT" worktree remove --force "$T"
echo "ab_base/ = $C"
