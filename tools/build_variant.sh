#!/bin/bash
# Build an A/B variant of the library: tools/build_variant.sh NAME "-DFLAG=1 ..."
# -> pl-vi-orbslam3_amd/variants/NAME/libplvi_frontend.so (select with PLVI_LIB=...).
set -e
cd "$(dirname "$0")/../pl-vi-orbslam3_amd"
make -s -j8 BUILD=variants/$1/build OUT=variants/$1/libplvi_frontend.so EXTRA="$2"
echo "PLVI_LIB=$(pwd)/variants/$1/libplvi_frontend.so"
