#!/bin/bash
# round 6: nt-policy stored-q CG as the default: A/B vs the split tail's x in Xc with nt,
# then the backbone / distributed-select / boundary GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/variant_ab.sh r06e main xnt || exit 1
bash tools/r06a_check.sh
