#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r06w_check.sh || exit 1
bash tools/r06x_check.sh
