#!/bin/bash
# Round 5: epilogue C-tile swap A/B (gpu_r05_cswz.sh), then the CTR tests and rehearsal
# with the autograd-free tower step (gpu_r05_ctr2.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_r05_cswz.sh && bash scripts/gpu_r05_ctr2.sh
