#!/bin/bash
# Round 5, cap and resume of the canopy Newton loop: the new and capped GPU
# tests, then an interleaved A/B of the cap on config #3, then the Fortran
# slot timed at 1 M columns and one driver-style bench line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05c}
mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread \
  -k "vege_cap or midloop or rccl or exhaustive or region_edges or engine_slot or single_call_bit_exact" > "$O/pytest_new.log" 2>&1
rc=$?; echo "new tests rc=$rc"; tail -3 "$O/pytest_new.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for k in 0 10 12 8 14 6; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --vege-cap $k > "$O/cap${k}_$rep.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench cap $k rc=$rc"; tail -3 "$O/cap${k}_$rep.log"; exit $rc; }
    python -c "import json; d=json.loads(open('$O/cap${k}_$rep.log').read().strip().splitlines()[-1]); print('cap $k rep $rep', round(d['value']/1e6,1), 'Mcs/s step_ms', round(d['roofline']['step_ms'],4))" | tee -a "$O/cap_ab.txt"
  done
done
timeout -k 10 300 python -u tools/drop_in_timing.py --ncol 1048576 --steps 20 --out "$O/dropin.json" > "$O/dropin.log" 2>&1
rc=$?; echo "drop-in timing rc=$rc"; tail -5 "$O/dropin.log"; [ $rc -eq 0 ] || exit $rc
