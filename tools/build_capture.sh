#!/bin/bash
# builds the graph-capture diagnostics (tools/capture_probe.hip, tools/capture_frame.cpp)
set -e
D=$(cd "$(dirname "$0")" && pwd)
mkdir -p $D/_build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -o $D/_build/capture_probe $D/capture_probe.hip
/opt/rocm/bin/hipcc -O1 -g -rdynamic -I$D/../include -o $D/_build/capture_frame $D/capture_frame.cpp \
  -L$D/../pl-vi-orbslam3_amd/lib -lplvi_frontend -Wl,-rpath,'$ORIGIN/../../pl-vi-orbslam3_amd/lib'
