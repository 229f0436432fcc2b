#!/bin/bash
# Per-phase counters of the step kernel.  The probe
# library lib_trunc.so (tools/build_variants.py "trunc": -DNMP_TRUNC_RUNTIME)
# returns from the column's step at phase mark NMP_TRUNC_AT (a run-time
# kernel argument, so nothing before the mark is optimised away); the
# difference between consecutive marks is one phase.  For each mark: a
# kernel-trace run (durations) and three PMC passes (<= 8 SQ counters each,
# --kernel-trace only) of a short bench.  tools/phase_counters.py turns the
# CSVs into profiles/r06/phase_counters.json.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${TAG:-phase_ctr}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export NOAHMP_ENGINE_LIB="$R/noahmp-1_amd/lib/variants/lib_trunc.so"
[ -f "$NOAHMP_ENGINE_LIB" ] || { echo "missing $NOAHMP_ENGINE_LIB"; exit 1; }
P1="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_WAVES"
P3="SQ_INSTS_SALU SQ_INSTS_VALU_INT32 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_WAVES"
BENCH="$R/bench.py --steps 4 --warmup 1 --period 4 --no-cpu-baseline ${BENCH_ARGS:-}"
for k in ${MARKS:-2 3 4 5 6 14 9 10 11 13 99}; do
  export NMP_TRUNC_AT=$k
  mkdir -p "$OUT/m$k"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/m$k/kt" -o run -- python3 $BENCH > "$OUT/m$k/kt.log" 2>&1 \
    || { echo "mark $k kt failed"; tail -3 "$OUT/m$k/kt.log"; exit 1; }
  for p in 1 2 3; do
    eval "C=\$P$p"
    timeout -k 10 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/m$k/p$p" -o run -- python3 $BENCH > "$OUT/m$k/p$p.log" 2>&1 \
      || { echo "mark $k pass $p failed"; tail -3 "$OUT/m$k/p$p.log"; exit 1; }
  done
  echo "mark $k done"
done
