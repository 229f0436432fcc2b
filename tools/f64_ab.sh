#!/bin/bash
# fp64 translation-unit flags: the parity file on the default library and on
# each variant, then configs #2 and #5 for the default and the variants.
# VARIANTS="f64ieee f64afn".  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-f64ab}; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
V="${VARIANTS:-f64ieee f64afn}"
for v in default $V; do
  if [ "$v" = default ]; then lib=""; else lib=$PWD/noahmp-1_amd/lib/variants/lib_$v.so; fi
  NOAHMP_ENGINE_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > "$OUT/parity_$v.log" 2>&1
  rc=$?; echo "parity $v rc=$rc: $(tail -1 $OUT/parity_$v.log)"; [ $rc -le 1 ] || exit $rc
done
CFG2="--kind casenml --ncol 65536 --precision 8"
CFG5="--kind global --ncol 1036800 --precision 8 --opt-veg 2 --dt 3600 --out-every 1 --forcing device"
for rep in 1 2; do
  for v in default $V; do
    if [ "$v" = default ]; then lib=""; else lib=$PWD/noahmp-1_amd/lib/variants/lib_$v.so; fi
    for c in 2 5; do
      if [ $c = 2 ]; then a=$CFG2; else a=$CFG5; fi
      NOAHMP_ENGINE_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 48 --warmup 4 $a > "$OUT/cfg${c}_${v}_$rep.json" 2>"$OUT/cfg${c}_${v}_$rep.err"
      rc=$?; [ $rc -eq 0 ] || { echo "cfg$c $v rc=$rc"; tail -3 "$OUT/cfg${c}_${v}_$rep.err"; exit $rc; }
      python -c "import json; d=json.load(open('$OUT/cfg${c}_${v}_$rep.json')); print('cfg$c $v $rep', round(d['value']/1e6,1), 'Mcs/s step_ms', round(d['roofline']['step_ms'],4))"
    done
  done
done
