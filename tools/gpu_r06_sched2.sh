#!/bin/bash
# r06: schedule options re-measured under one growth task per wave (ORB chain the
# busier): ORB pyramid level by level at 3072, ORB after the LSD prep, growth
# without the blur gate, ORB stream at normal priority
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
CONFIGS="base|-|-;pyrlw|-|PLVI_PYR_LEVELWISE=4096;orbprep2|-|PLVI_ORB_AFTER_PREP=2;nogate|-|PLVI_GROW_AFTER_BLUR=0;orblow|-|PLVI_ORB_PRIO=0" REPS=2 bash tools/ab_mix.sh
