#!/bin/bash
# r06: wave priorities after one growth task per wave made the ORB chain the
# longer one again: growth waves at s_setprio 1 / 0 (default 3), ORB waves at 3
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
CONFIGS="base|-|-;gp1|gp1|-;gp0|gp0|-;op3|op3|-" REPS=2 bash tools/ab_mix.sh
