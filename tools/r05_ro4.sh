#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/r05_ro3.sh r05_ro4 || exit $?
bash $R/tools/r05_mixed_ab.sh r05_mixed_ab2 || exit $?
echo all_done
