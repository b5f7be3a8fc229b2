#!/bin/bash
# GPU box: headline kernel-trace timeline (per-query GPU time vs wall) on the current tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
STEPS=10 TAIL=60 TL=6 bash tools/gpu_prof_headline.sh || exit 1
rm -rf gpurun_out/profh
