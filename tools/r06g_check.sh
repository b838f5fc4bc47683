#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R06A_TAG=r06g bash tools/r06a_check.sh || exit 1
bash tools/r06f_jac_ab.sh
