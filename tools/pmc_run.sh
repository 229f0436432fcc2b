#!/bin/bash
# PMC passes (GPU box): HBM bytes of the engine kernel and of the calibration
# copy, one counter per pass, --kernel-trace only (no sys/runtime traces).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${TAG:-pmc}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
[ -x "$R/tools/calib_copy" ] || hipcc -O3 --offload-arch=gfx950 -o "$R/tools/calib_copy" "$R/tools/calib_copy.hip" || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 180 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/calib_$C" -o run -- "$R/tools/calib_copy" 4194304 3 > "$OUT/calib_$C.log" 2>&1
  rc=$?; echo "calib $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/bench_$C" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench_$C.log" 2>&1
  rc=$?; echo "bench $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
if [ "${VALU:-1}" = 1 ]; then
  # two SQ passes (at most 8 SQ counters each): the VALU total, issue activity
  # and memory instructions, then the VALU instruction classes the bench line's
  # cycle-weighted VALU fraction needs (bench.py valu_weighted)
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F64 --kernel-trace --output-format csv -d "$OUT/bench_SQ" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench_SQ.log" 2>&1
  rc=$?; echo "bench SQ rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_WAVES --kernel-trace --output-format csv -d "$OUT/bench_SQ2" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench_SQ2.log" 2>&1
  rc=$?; echo "bench SQ2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  # lane utilisation of the VALU: thread-cycles of VALU
  # work over 64 x the waves' VALU cycles, from one pass
  timeout -k 10 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d "$OUT/bench_SQ3" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench_SQ3.log" 2>&1
  rc=$?; echo "bench SQ3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
find "$OUT" -name "*.csv" | head -20
