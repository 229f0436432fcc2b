#!/bin/bash
# Config #2 (65,536 replicated case.nml columns, fp64 / fp32): streams, with the
# automatic kernel choice (half-occupancy kernel for small launches), and the
# config #3 headline.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-smalln}; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
for cfg in 8_1 8_2 4_1 4_2; do
  p=${cfg%_*}; s=${cfg#*_}
  timeout -k 10 200 python bench.py --no-cpu-baseline --ncol 65536 --kind casenml --precision $p --steps 96 --streams $s > "$OUT/b_$cfg.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg rc=$rc"; tail -3 "$OUT/b_$cfg.log"; exit $rc; }
  python -c "import json; d=json.loads(open('$OUT/b_$cfg.log').read().strip().splitlines()[-1]); print('precision $p streams $s', round(d['value']/1e6,1), 'Mcs/s step_ms', round(d['roofline']['step_ms'],4), 'frac', round(d['roofline']['frac'],4))"
done
timeout -k 10 200 python bench.py --no-cpu-baseline > "$OUT/b_cfg3.log" 2>&1 || exit 1
python -c "import json; d=json.loads(open('$OUT/b_cfg3.log').read().strip().splitlines()[-1]); print('config #3', round(d['value']/1e6,1), 'Mcs/s')"
