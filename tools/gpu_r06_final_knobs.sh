#!/bin/bash
# r06 (final HEAD): octree LDS stage 1024 and ORB after the LSD prep, env-only A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
CONFIGS="base|-|-;oct1024|-|PLVI_ORB_OCT_LDS=1024;prep2|-|PLVI_ORB_AFTER_PREP=2" REPS=3 bash tools/ab_mix.sh
