#!/bin/bash
# r06: counter padding A/B, in-tree (padded) first in each pair
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
CONFIGS="pad32|-|-;pad1|pad1|-" REPS=3 bash tools/ab_mix.sh
