#!/bin/bash
# Build an A/B variant of the engine library into pbccs_amd/_lib_ab/ (loaded with PBCCS_LIB by the
# tools/gpu_steps.sh ab_lib step).  The variant is the working tree's csrc with some files taken from a git
# revision:  tools/build_ab.sh REV file.hip [file.hpp ...]   (paths relative to pbccs_amd/csrc)
# Extra compiler flags for the variant: AB_FLAGS="-DFOO=1" tools/build_ab.sh HEAD; another output directory: AB_OUT=...
# (the occupancy build: AB_FLAGS="-DPBCCS_WAVE_STAMPS=1" AB_OUT=pbccs_amd/_lib_occ tools/build_ab.sh HEAD)
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:-HEAD}; shift || true
T=$(mktemp -d /tmp/pbccs_ab.XXXXXX)
mkdir -p "$T/pbccs_amd"
cp -r "$REPO/include" "$T/include"
cp -r "$REPO/pbccs_amd/csrc" "$T/pbccs_amd/csrc"
for f in "$@"; do git -C "$REPO" show "$REV:pbccs_amd/csrc/$f" > "$T/pbccs_amd/csrc/$f"; done
F="-std=c++17 -O3 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function -fno-gpu-flush-denormals-to-zero --offload-arch=gfx950 ${AB_FLAGS:-}"
OUTD=${AB_OUT:-pbccs_amd/_lib_ab}
make -s -j8 -C "$T/pbccs_amd/csrc" HIPFLAGS="$F" OUT="$REPO/$OUTD" OBJ="$T/build"
rm -rf "$T"
echo "built $OUTD/libpbccs_amd.so (csrc with $* from $REV)"
