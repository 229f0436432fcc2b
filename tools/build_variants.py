"""Build tuning variants of the engine library into noahmp-1_amd/lib/variants/."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import noahmp_pkg  # noqa: E402,F401
from noahmp_amd import build  # noqa: E402

VARIANTS = {
    "base": (),
    "w2": ("-DNMP_WAVES_PER_EU=2",),
    "outline": ("-DNMP_MATH_OUTLINE",),
    "outline_w2": ("-DNMP_MATH_OUTLINE", "-DNMP_WAVES_PER_EU=2"),
    "w4": ("-DNMP_WAVES_PER_EU=4",),
    "w1": ("-DNMP_WAVES_PER_EU=1",),
    "w3": ("-DNMP_WAVES_PER_EU=3",),
    "phase": ("-DNMP_PHASE_TIMING",),
    "phase_nopf": ("-DNMP_PHASE_TIMING", "-DNMP_PREFETCH=0"),
    "nopf": ("-DNMP_PREFETCH=0",),
    "nt0": ("-DNMP_NT=0",),
    "u_l2": ("-DNMP_LOOP2_UNROLL=5",),
    "u_bare": ("-DNMP_BARE_UNROLL=5",),
    "u_both": ("-DNMP_LOOP2_UNROLL=5", "-DNMP_BARE_UNROLL=5"),
    "pf1": ("-DNMP_PREFETCH=1",),
    # fp64 translation unit flags (the fp32 kernels unchanged)
    "f64ieee": {"f64": []},
    "f64afn": {"f64": ["-freciprocal-math", "-fapprox-func"]},
    "pf2": ("-DNMP_PREFETCH=2",),
    "b128": ("-DNMP_BLOCK=128",),
    "b64": ("-DNMP_BLOCK=64",),
    "b512": ("-DNMP_BLOCK=512",),
    "k6": ("-DNMP_VEGE_K=6",),
    "k10": ("-DNMP_VEGE_K=10",),
    "k12": ("-DNMP_VEGE_K=12",),
    "k20": ("-DNMP_VEGE_K=20",),
    "k20lds": ("-DNMP_VEGE_K=20", "-DNMP_LDS_PAD=32768"),
    "k12off": ("-DNMP_VEGE_K=12", "-DNMP_VPOOL_OFF"),
    "w4_b128": ("-DNMP_WAVES_PER_EU=4", "-DNMP_BLOCK=128"),
    "w4_b64": ("-DNMP_WAVES_PER_EU=4", "-DNMP_BLOCK=64"),
    "w5": ("-DNMP_WAVES_PER_EU=5",),
    "d1": ("-DNMP_WAVES_PER_EU_F64=1",),
    "w2_d1": ("-DNMP_WAVES_PER_EU=2", "-DNMP_WAVES_PER_EU_F64=1"),
    # round 6: the soil-water sub-steps' divisions on IEEE only (A/B of NMP_SOIL_DIV)
    "soildiv0": {"f32": ["-DNMP_SOIL_DIV=0"]},
    # per-phase truncation at a run-time mark (tools/phase_counters.sh)
    "trunc": ("-DNMP_TRUNC_RUNTIME",),
    "en_w4": ("-DNMP_TRUNC_ENERGY",),
    "en_w5": ("-DNMP_TRUNC_ENERGY", "-DNMP_WAVES_PER_EU=5"),
    "en_w3": ("-DNMP_TRUNC_ENERGY", "-DNMP_WAVES_PER_EU=3"),
    "en_w6": ("-DNMP_TRUNC_ENERGY", "-DNMP_WAVES_PER_EU=6"),
    "en_w8": ("-DNMP_TRUNC_ENERGY", "-DNMP_WAVES_PER_EU=8"),
    "d2": ("-DNMP_WAVES_PER_EU_F64=2",),
    "s_maxilp": ("-mllvm", "-amdgpu-sched-strategy=max-ilp"),
    "s_memclause": ("-mllvm", "-amdgpu-sched-strategy=max-memory-clause"),
    "s_itminreg": ("-mllvm", "-amdgpu-sched-strategy=iterative-minreg"),
    "s_itilp": ("-mllvm", "-amdgpu-sched-strategy=iterative-ilp"),
    "s_nomisched": ("-mllvm", "-enable-misched=false"),
    "s_postup": ("-mllvm", "-misched-postra-direction=bottomup"),
    "d3": ("-DNMP_WAVES_PER_EU_F64=3",),
    "mlicm": ("-mllvm", "-disable-machine-licm=false"),
    "w4_mlicm": ("-DNMP_WAVES_PER_EU=4", "-mllvm", "-disable-machine-licm=false"),
    "split_speed": ("-mllvm", "-split-spill-mode=speed"),
    "split_size": ("-mllvm", "-split-spill-mode=size"),
    "rptrack": ("-mllvm", "-amdgpu-use-amdgpu-trackers"),
    "dce_ra": ("-mllvm", "-amdgpu-dce-in-ra"),
    "nounclust": ("-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule"),
    "relaxocc": ("-mllvm", "-amdgpu-schedule-relaxed-occupancy"),
    "outline_w3": ("-DNMP_MATH_OUTLINE", "-DNMP_WAVES_PER_EU=3"),
    "lds_work": ("-DNMP_LDS_WORK",),
    "lds_state": ("-DNMP_LDS_STATE",),
    # timing probes only (NOT bit-exact): upper bounds of what faster division
    # / sqrt sequences could save
    "nocrdiv": ("-fno-hip-fp32-correctly-rounded-divide-sqrt",),
    "fdiv9": {"f32": ["-DNMP_F32_DIV=9"]},
    "cr9": {"f32": ["-DNMP_F32_DIV=1"]},
    "ldswait0": {"f32": ["-DNMP_LDS_EXPLICIT_WAIT=0"]},
    "dgetbr": ("-DNMP_DGET_BRANCHY",),
    "fdiv7": {"f32": ["-DNMP_F32_DIV=7"]},
    # round 4: the canopy loop with IEEE division only (before the range-proved
    # short division became the default)
    "vd0": {"f32": ["-DNMP_VEGE_DIV=0"]},
    "bare0": {"f32": ["-DNMP_BARE_DIV=0"]},
    # tables read from global memory (no per-workgroup LDS staging), smaller blocks
    "noshare": {"f32": ["-DNMP_DIV_NOSHARE"]},
    "vdnofb": {"f32": ["-DNMP_VD_NOFALLBACK"]},
    # domain checks dropped by bit (timing probes only, not exact in general)
    "dm0_3": {"f32": ["-DNMP_DOM_MASK=0xfffffff0u"]},
    "dm4_8": {"f32": ["-DNMP_DOM_MASK=0xfffffe0fu"]},
    "dm9_14": {"f32": ["-DNMP_DOM_MASK=0xffff81ffu"]},
    "dmwin": {"f32": ["-DNMP_DOM_MASK=0xfff0ffffu"]},
    "pg": ("-DNMP_PARAMS_GLOBAL",),
    "pg128": ("-DNMP_PARAMS_GLOBAL", "-DNMP_BLOCK=128"),
    "pg64": ("-DNMP_PARAMS_GLOBAL", "-DNMP_BLOCK=64"),
    # the default build plus a device counter of lanes that re-ran the canopy
    # loop with IEEE division (nmp_debug_fallback_count)
    "fbcount": {"f32": ["-DNMP_COUNT_FALLBACK"]},
    # timing probes of the range-checked canopy division (not exact in general)
    "vdnodom": {"f32": ["-DNMP_VD_NODOMAIN"]},
    "vdnowin": {"f32": ["-DNMP_VD_NOWIN"]},
    "vdallfast": {"f32": ["-DNMP_VD_ALLFAST"]},
    "vdnone": {"f32": ["-DNMP_VD_NODOMAIN", "-DNMP_VD_NOWIN", "-DNMP_VD_ALLFAST"]},
    # round 6: CTR, TR, DTV (bit 0) and bare DTG (bit 1) on DivFast32 with
    # per-lane numerator windows (exact: a lane outside re-runs with IEEE)
    "vdchk": {"f32": ["-DNMP_VD_CHECKED=3"]},
    "vdchk1": {"f32": ["-DNMP_VD_CHECKED=1"]},
    "vdchk2": {"f32": ["-DNMP_VD_CHECKED=2"]},
    "vdchk_fb": {"f32": ["-DNMP_VD_CHECKED=3", "-DNMP_COUNT_FALLBACK"]},
    "nopeel": ("-DNMP_VEGE_NOPEEL",),
    "vu2": ("-DNMP_VEGE_UNROLL=2",),
    "vu3": ("-DNMP_VEGE_UNROLL=3",),
    "pinnv": ("-DNMP_PIN_NONVOLATILE",),
    "dvnoguard": ("-DNMP_F64_DV_NOGUARD",),
    "dvieee": ("-DNMP_F64_IEEE_DIV",),
    "ocmlpow": ("-DNMP_F64_OCML_POW",),
    "noslp": ("-fno-slp-vectorize",),
    "nolpre": ("-mllvm", "-enable-load-pre=false"),
    "nopre": ("-mllvm", "-enable-pre=false"),
    "nounroll": ("-fno-unroll-loops",),
    "nopostmis": ("-mllvm", "-enable-post-misched=false"),
    "nosink": ("-mllvm", "-simplifycfg-sink-common=false"),
    "nohoist": ("-mllvm", "-simplifycfg-hoist-common=false"),
    "phifold8": ("-mllvm", "-two-entry-phi-node-folding-threshold=8"),
    "exhaust": ("-mllvm", "-exhaustive-register-search"),
    "defer": ("-mllvm", "-enable-deferred-spilling"),
    "nomcse": ("-mllvm", "-disable-machine-cse"),
    # the fp64 translation unit alone without MachineCSE
    "nomcse64": {"f64": ["-mllvm", "-disable-machine-cse"]},
    "dbg64": {"f64": ["-DNMP_DEBUG_DUMP"]},
    "nomcse64_dbg": {"f64": ["-mllvm", "-disable-machine-cse", "-DNMP_DEBUG_DUMP"]},
    "notaildup": ("-mllvm", "-disable-tail-duplicate", "-mllvm", "-disable-early-taildup"),
    "gvnsink": ("-mllvm", "-enable-gvn-sink"),
    "nolsv": ("-mllvm", "-amdgpu-load-store-vectorizer=false"),
    # fp32 translation unit only
    "notaildup32": {"f32": ["-mllvm", "-disable-tail-duplicate", "-mllvm", "-disable-early-taildup"]},
    "nosink32": {"f32": ["-mllvm", "-simplifycfg-sink-common=false"]},
    "phifold1_32": {"f32": ["-mllvm", "-two-entry-phi-node-folding-threshold=1"]},
    "specoff32": {"f32": ["-mllvm", "-speculate-one-expensive-inst=false"]},
    "o2": ("-O2",),
    # probes of the soil-layer math sharing (results identical either way)
    "nopowpair": ("-DNMP_POW_PAIR=0",),
    "nounfrozen": ("-DNMP_UNFROZEN_FAST=0",),
    "no2mskip": ("-DNMP_SKIP_2M=0",),
    "gmbl": ("-DNMP_GM_BRANCHLESS=1",),
    "stfast": {"f32": ["-DNMP_STOMATA_FASTDIV"]},
    "sqrtieee": {"f32": ["-DNMP_SQRT_SHORT=0"]},
    # round-4 re-sweep on the fp32 translation unit
    "bu1": {"f32": ["-DNMP_BARE_UNROLL=1"]},
    "bu3": {"f32": ["-DNMP_BARE_UNROLL=3"]},
    "vu2_32": {"f32": ["-DNMP_VEGE_UNROLL=2"]},
    "maxilp32": {"f32": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]},
    "exhaust32": {"f32": ["-mllvm", "-exhaustive-register-search"]},
    "gcprio32": {"f32": ["-mllvm", "-greedy-regclass-priority-trumps-globalness=true"]},
    "nopostmis32": {"f32": ["-mllvm", "-enable-post-misched=false"]},
    "w5_32": {"f32": ["-DNMP_WAVES_PER_EU=5"]},
    "gcprio": ("-mllvm", "-greedy-regclass-priority-trumps-globalness=true"),
    # per-wave start/end records (tools/wave_timeline.py)
    "wt": ("-DNMP_WAVE_TIMING",),
    "wt_b128": ("-DNMP_WAVE_TIMING", "-DNMP_BLOCK=128", "-DNMP_PREFETCH=0"),
    "wt_b64": ("-DNMP_WAVE_TIMING", "-DNMP_BLOCK=64", "-DNMP_PREFETCH=0"),
    "b128_nopf": ("-DNMP_BLOCK=128", "-DNMP_PREFETCH=0"),
    "b64_nopf": ("-DNMP_BLOCK=64", "-DNMP_PREFETCH=0"),
    # round 5: fp64 exp with an Estrin polynomial (shorter dependent chain,
    # config #2's one wave per SIMD; sflx_math.h exp_estrin)
    "f64estrin": {"f64": ["-DNMP_F64_EXP_ESTRIN=1"]},
    # timing probes (results wrong for the capped lanes): the canopy Newton
    # loop capped at K iterations, capped lanes leaving the step -- the main
    # launch of a cap-and-resume split (tools/cap_resume_model.py)
    # 64-bit per-lane column pointers (the addressing before round 5's 32-bit offsets)
    "off64": ("-DNMP_OFF32=0",),
    "off32": ("-DNMP_OFF32=1",),
    # the SLP vectorizer back on (the base flags' -fno-slp-vectorize overridden)
    "slp": ("-fslp-vectorize",),
    # field bases recomputed per access (no per-field SGPR bases to spill)
    "off32r": ("-DNMP_OFF32=2",),
    "off32r_w5": ("-DNMP_OFF32=2", "-DNMP_WAVES_PER_EU=5"),
    # array bases re-read from the kernel-argument segment per access
    "off32k": ("-DNMP_OFF32=3",),
    # flux / water phase fields loaded a phase early (NMP_EARLY_LOADS bits)
    # the fp64 small kernels without MachineLICM (the build before the split)
    "f64s_nolicm": {"f64s": ["-mllvm", "-disable-machine-licm"]},
    # machine-scheduler strategies for the fp32 unit
    "s_ilp": {"f32": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]},
    "s_itilp": {"f32": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]},
    "s_memcl": {"f32": ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"]},
    # (timing probe, not exact) the soil-water sub-steps' divisions as a * rcp(b)
    # (needs tools/patches/soil_div_probe.patch applied)
    "soildiv": {"f32": ["-DNMP_SOIL_DIV_PROBE"]},
    # sunlit and shaded stomata solves interleaved (needs tools/patches/stomata_pair.patch)
    "stpair": {"f32": ["-DNMP_STOMATA_PAIR=1"]},
    "el1": {"f32": ["-DNMP_EARLY_LOADS=1"]},
    "el2": {"f32": ["-DNMP_EARLY_LOADS=2"]},
    "el3": {"f32": ["-DNMP_EARLY_LOADS=3"]},
    # base flags re-checked once the spills were gone: MachineLICM and GVN-PRE
    # back on ("drop": flag pairs removed from build.FLAGS)
    "licm": {"drop": [("-mllvm", "-disable-machine-licm")]},
    "pre": {"drop": [("-mllvm", "-enable-pre=false")]},
}
if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    vdir = os.path.join(build.LIB_DIR, "variants")
    base_flags = list(build.FLAGS)

    def drop(flags, seqs):
        out, i = [], 0
        while i < len(flags):
            for q in seqs:
                if tuple(flags[i:i + len(q)]) == tuple(q):
                    i += len(q)
                    break
            else:
                out.append(flags[i])
                i += 1
        return out

    def one(n):
        v = VARIANTS[n]
        if isinstance(v, dict) and "drop" in v:  # run alone: build.FLAGS patched
            build.FLAGS = drop(base_flags, v["drop"])
            sf = {k: drop(f, v["drop"]) for k, f in build.SOURCE_FLAGS.items()}
            try:
                return build.build(force=True, verbose=False, out=os.path.join(vdir, f"lib_{n}.so"),
                                   source_flags=sf)
            finally:
                build.FLAGS = base_flags
        if isinstance(v, dict):  # per-source flags: {"extra": (...), "f64": [...]}
            sf = dict(build.SOURCE_FLAGS)
            if "f64" in v:
                sf["sflx_kernel_f64.hip"] = list(sf["sflx_kernel_f64.hip"]) + list(v["f64"])
            if "f64s" in v:  # extra flags for the fp64 small-kernel unit only
                sf["sflx_kernel_f64s.hip"] = list(sf["sflx_kernel_f64s.hip"]) + list(v["f64s"])
            if "f32" in v:  # extra flags for the fp32 translation unit only
                sf["sflx_kernel.hip"] = list(sf["sflx_kernel.hip"]) + list(v["f32"])
            return build.build(force=True, verbose=False, out=os.path.join(vdir, f"lib_{n}.so"),
                               extra=tuple(v.get("extra", ())), source_flags=sf,
                               check_asm=not n.startswith("nomcse"))
        return build.build(force=True, verbose=False, out=os.path.join(vdir, f"lib_{n}.so"), extra=v,
                           check_asm=not n.startswith("nomcse"))
    solo = [n for n in names if isinstance(VARIANTS[n], dict) and "drop" in VARIANTS[n]]
    with ThreadPoolExecutor(2) as ex:
        list(ex.map(one, [n for n in names if n not in solo]))
    for n in solo:
        one(n)
    print("built", names)
