#!/bin/bash
# r03i: rocprofv3 evidence for the headline kernel (tools/profile.sh) and bench.py's other
# BASELINE configs (tools/profile_configs.sh) on the current build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/profile.sh || exit 1
bash tools/profile_configs.sh || exit 1
