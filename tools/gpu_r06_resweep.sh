#!/bin/bash
# r06: schedule knobs re-measured after the candidate-list ORB middle (the
# line chain is the longer one again): growth tasks per wave, Sobel pyramid
# placement, octave-split growth
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
CONFIGS="base|-|-;tpw1|-|PLVI_GROW_TPW=1;sobelafter|-|PLVI_SOBEL_AFTER_GROW=1;split|-|PLVI_GROW_SPLIT=1;tpw1split|-|PLVI_GROW_TPW=1 PLVI_GROW_SPLIT=1" REPS=2 bash tools/ab_mix.sh
