#!/bin/bash
# Closing pass after the julian range check: evidence pass, configs, the year.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r03final3 bash tools/final_r03.sh || exit $?
TAG=configs_r03b STEPS=48 bash tools/configs.sh || exit $?
TAG=year3 bash tools/year_run.sh
