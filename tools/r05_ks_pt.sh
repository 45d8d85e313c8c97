#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/r05_ksweep.sh r05_ksweep || exit $?
bash $R/tools/r05_puct_trace.sh r05_puct_trace || exit $?
echo all_done
