#!/bin/bash
# Build an A/B variant of libgsr.so from the working tree with extra defines
# (development): bash tools/build_variant.sh NAME "-DGSR_X=0 ..." ["FLAGS_file=... (make variables)"]  ->  ab_libs/NAME.so
set -e
NAME=$1; DEFS=$2; MAKEVARS=$3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/gsr_variant_$NAME
rm -rf $W && mkdir -p $W/pkg $W/include
cp -r $ROOT/geometry-grounded-gaussian-splatting_amd/csrc $ROOT/geometry-grounded-gaussian-splatting_amd/Makefile $W/pkg/
cp $ROOT/include/*.h $W/include/
mkdir -p $W/pkg/diff_gaussian_rasterization
make -s -C $W/pkg -j8 HIPFLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -Wall -Wno-unused-result -I../include -Icsrc $DEFS" $MAKEVARS > $W/build.log 2>&1
mkdir -p $ROOT/ab_libs
cp $W/pkg/diff_gaussian_rasterization/libgsr.so $ROOT/ab_libs/$NAME.so
echo "ab_libs/$NAME.so ($DEFS)"
