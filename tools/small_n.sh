#!/bin/bash
# Config #2 (65,536 replicated case.nml columns, fp64): columns per wave x streams,
# plus the new cpw tests and the config #3 headline (auto cpw must stay 64).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-smalln}; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "cols_per_wave" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for cfg in 64_2 64_1 0_1 0_2 32_1 16_1 16_2 8_1 8_2; do
  c=${cfg%_*}; s=${cfg#*_}
  timeout -k 10 200 python bench.py --no-cpu-baseline --ncol 65536 --kind casenml --precision 8 --steps 96 --cpw $c --streams $s > "$OUT/b_$cfg.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg rc=$rc"; tail -3 "$OUT/b_$cfg.log"; exit $rc; }
  python -c "import json; d=json.loads(open('$OUT/b_$cfg.log').read().strip().splitlines()[-1]); print('cpw $c streams $s', round(d['value']/1e6,1), 'Mcs/s step_ms', round(d['roofline']['step_ms'],4), 'frac', round(d['roofline']['frac'],4))"
done
timeout -k 10 200 python bench.py --no-cpu-baseline > "$OUT/b_cfg3.log" 2>&1 || exit 1
python -c "import json; d=json.loads(open('$OUT/b_cfg3.log').read().strip().splitlines()[-1]); print('config #3', round(d['value']/1e6,1), 'Mcs/s')"
