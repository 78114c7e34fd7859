#!/bin/bash
# Build a tuning variant of libge.so with extra -D flags (kernel knobs such as
# GE_TILE_CAP, GE_TILE_ROWS, GE_ROWS_MINBLOCKS, GE_BAR_ORDER) into
# graph-embed_amd/variants/NAME/.  ONLY="ge_fa ge_faml" recompiles just those
# sources with the flags and links the main build's objects for the rest.
# Load it with GE_LIB_PATH=graph-embed_amd/variants/NAME/libge.so (tuning only).
# Do not edit the sources while a variant builds: hipcc reads them once per pass.
set -e
NAME=$1; shift
HERE=$(cd "$(dirname "$0")/../graph-embed_amd" && pwd)
OUT=$HERE/variants/$NAME
mkdir -p $OUT
make -s -C $HERE >/dev/null
HIP_OBJ=""
for f in $HERE/csrc/*.hip; do
  b=$(basename $f .hip)
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $b "* ]]; then
    HIP_OBJ="$HIP_OBJ $HERE/build/$b.o"
    continue
  fi
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
    -munsafe-fp-atomics -I$HERE/../include -I$HERE/csrc "$@" -c $f -o $OUT/$b.o &
  HIP_OBJ="$HIP_OBJ $OUT/$b.o"
done
wait
CPP_OBJ=$(for f in $HERE/csrc/*.cpp; do echo $HERE/build/$(basename $f .cpp).o; done)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT/libge.so $HIP_OBJ $CPP_OBJ \
  $(g++ -print-file-name=libgomp.so) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libge.so
rm -f $OUT/*.o
echo $OUT/libge.so
