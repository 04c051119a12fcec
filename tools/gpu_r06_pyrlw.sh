#!/bin/bash
# r06: the ORB pyramid level by level at 3072 frames too (PLVI_PYR_LEVELWISE=4096)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
CONFIGS="base|-|-;pyrlw|-|PLVI_PYR_LEVELWISE=4096" REPS=3 bash tools/ab_mix.sh
