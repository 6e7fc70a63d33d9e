#!/bin/bash
# Build libmosaic_gpu.so from a git revision into build/variants/NAME (for A/B runs
# against the working tree): tools/ab_build.sh REV NAME
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/mgpu_ab_$NAME
rm -rf $W; git -C $ROOT worktree prune; git -C $ROOT worktree add -f --detach $W $REV > /dev/null
mkdir -p $ROOT/build/variants/$NAME
make -s -C $W/mosaic_amd/csrc OUT=$ROOT/build/variants/$NAME/libmosaic_gpu.so $ROOT/build/variants/$NAME/libmosaic_gpu.so
git -C $ROOT worktree remove --force $W
