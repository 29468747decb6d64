#!/bin/bash
# Build the engine library as of git revision REV into OUTDIR (relative to the repo root), for bisecting a
# behaviour change on the GPU box (PBCCS_LIB=OUTDIR/libpbccs_amd.so).  Usage: tools/build_rev.sh REV OUTDIR
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; OUTDIR=$2
T=$(mktemp -d /tmp/pbccs_rev.XXXXXX)
git -C "$REPO" archive "$REV" include pbccs_amd/csrc | tar -x -C "$T"
make -s -j8 -C "$T/pbccs_amd/csrc" OUT="$REPO/$OUTDIR" OBJ="$T/build"
rm -rf "$T"
echo "built $OUTDIR/libpbccs_amd.so at $REV"
