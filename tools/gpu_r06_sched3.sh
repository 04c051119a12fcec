#!/bin/bash
# r06: ORB stream at normal priority (PLVI_ORB_PRIO=0) and ORB after the LSD prep
# for every batch (PLVI_ORB_AFTER_PREP=2), alone and together
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
CONFIGS="base|-|-;orblow|-|PLVI_ORB_PRIO=0;orbprep2|-|PLVI_ORB_AFTER_PREP=2;both|-|PLVI_ORB_PRIO=0 PLVI_ORB_AFTER_PREP=2" REPS=3 bash tools/ab_mix.sh
