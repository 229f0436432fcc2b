#!/bin/bash
# Round-3 closing pass on the final sources: the evidence pass (tools/final_r03.sh:
# tests, smoke, PMC, kernel trace, bench lines) and the other BASELINE configs.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r03final2 bash tools/final_r03.sh || exit $?
TAG=configs_r03 STEPS=48 bash tools/configs.sh
