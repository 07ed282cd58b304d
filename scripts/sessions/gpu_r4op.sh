#!/bin/bash
# Round-4 sessions O + P in one call: the pages-per-instruction probe (P), then the driver's bench command
# with the trio per upload form (O).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
bash scripts/sessions/gpu_r4p.sh && bash scripts/sessions/gpu_r4o.sh
