#!/bin/bash
# scripts/ab_rev.sh REV NAME -- libmijpeg.so built from git revision REV (a
# temporary worktree) as ab/libmijpeg_NAME.so, the baseline arm of scripts/ab.sh
set -e
cd "$(dirname "$0")/.."
wt=/tmp/mij_rev_$2
rm -rf $wt; git worktree prune
git worktree add -f --detach $wt $1 > /dev/null
make -s -C $wt/jpeg-encoder-decoder_amd libmijpeg.so 2> /dev/null
mkdir -p ab
cp $wt/jpeg-encoder-decoder_amd/libmijpeg.so ab/libmijpeg_$2.so
git worktree remove --force $wt
echo "ab/libmijpeg_$2.so"
