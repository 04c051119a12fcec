#!/bin/bash
# r06: describe pipeline A/B, second box, variant first in each pair
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
CONFIGS="descpipe|descpipe|-;base|-|-" REPS=4 bash tools/ab_mix.sh
