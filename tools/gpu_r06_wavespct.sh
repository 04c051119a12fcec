#!/bin/bash
# r06: large-batch growth with a fraction of its tasks doubled up per wave
# (PLVI_GROW_WAVES_PCT): parity at 3072 frames via the bench's oracle check, headline A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
CONFIGS="tpw1|-|-;p80|-|PLVI_GROW_WAVES_PCT=80;p67|-|PLVI_GROW_WAVES_PCT=67;tpw2|-|PLVI_GROW_TPW=0" REPS=2 bash tools/ab_mix.sh
