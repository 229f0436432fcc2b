#!/bin/bash
# Round-4 evidence pass on the committed sources: tests, smoke, PMC traffic and
# VALU classes, kernel trace, bench lines, distributed rehearsals, the other
# BASELINE configs (config #4 whole on one GPU included).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r04ev} bash tools/final_r04.sh || exit $?
TAG=${TAG:-r04ev}_configs STEPS=48 bash tools/configs.sh || exit $?
