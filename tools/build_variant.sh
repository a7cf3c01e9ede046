#!/bin/bash
# A/B builds of one source file: compile csrc/$FILE with extra -D flags and link it with the
# in-tree objects of every other file into ab/$NAME.so (timed on the GPU box through
# DH_LIB_PATH=ab/$NAME.so).  Usage: FILE=gemm_lnch.hip bash tools/build_variant.sh NAME "-DX=1 ..."
# (REV=<git rev>: that revision's version of the file instead of the working tree's)
set -e
cd "$(dirname "$0")/.."
NAME=$1; FLAGS=$2; FILE=${FILE:-gemm_lnch.hip}
python -c "from deephall_amd import _build; _build.build()" > /dev/null
mkdir -p ab build/ab
OBJ=build/ab/$NAME.$FILE.o
EXTRA=""; { [ "$FILE" = "gemm_x6.hip" ] || [ "$FILE" = "gemm_lnch.hip" ]; } && EXTRA="-fno-slp-vectorize"
SRC=deephall_amd/csrc/$FILE
if [ -n "$REV" ]; then SRC=deephall_amd/csrc/_rev_$FILE; git show $REV:deephall_amd/csrc/$FILE > $SRC; fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I include $EXTRA $FLAGS \
  -c $SRC -o $OBJ
[ -n "$REV" ] && rm -f $SRC
# the objects of the current link (build/gfx950/link.manifest), not a glob that would pick up
# stale objects of deleted sources
OBJS=$(grep -v "^$FILE.o$" build/gfx950/link.manifest | sed 's#^#build/gfx950/#')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab/$NAME.so $OBJS $OBJ
echo "built ab/$NAME.so ($FLAGS)"
