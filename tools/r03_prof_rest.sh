#!/bin/bash
# r03 final: rocprofv3 kernel stats + PMC of cfg1, cfg2, cfg4 at HEAD (tools/r03_prof.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT
CFGS="1 2 4" bash $R/tools/r03_prof.sh ${1:-r03_prof_rest}/prof || exit 1
