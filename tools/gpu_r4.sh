#!/bin/bash
# Round 4 GPU pass: the suite + smoke, then the team-width A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r4a.sh && bash tools/gpu_r4b.sh
