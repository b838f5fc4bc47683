#!/bin/bash
# round 6: stored-q CG (now the default) against its tuning variants and the old form
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/variant_ab.sh ${1:-r06c} ${@:2}
