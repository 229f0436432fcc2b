#!/bin/bash
# Round 5, first GPU pass: the new tests (mid-loop fallback probe, exhaustive
# short sqrt, division edges, RCCL gather on one GPU, fallback x diag level),
# the Fortran slot timed at 1 M columns, then the full GPU suite and a bench line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05a}
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread \
  -k "midloop or rccl or exhaustive or region_edges or fallback or engine_slot" > "$O/pytest_new.log" 2>&1
rc=$?; echo "new tests rc=$rc"; tail -3 "$O/pytest_new.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/drop_in_timing.py --ncol 1048576 --steps 20 --out "$O/dropin.json" > "$O/dropin.log" 2>&1
rc=$?; echo "drop-in timing rc=$rc"; cat "$O/dropin.log" | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > "$O/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 400 "$O/bench.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_all.log" 2>&1
rc=$?; echo "all tests rc=$rc"; tail -3 "$O/pytest_all.log"; exit $rc
