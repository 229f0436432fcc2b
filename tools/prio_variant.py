"""Build a timing variant of the engine with wave issue priority raised for
the canopy Newton loop's stragglers (not a product build).

A wave whose lanes are still iterating at iteration K of the vege_flux loop
(func.f90:2744-2877) sets its issue priority to P (`s_setprio`, a scalar
instruction: it takes effect for the whole wave whatever its lane mask) and
drops back to 0 after the loop.  Rationale: a workgroup holds its slot until
its slowest wave ends, so letting the long waves issue first on their SIMD
shortens the tail in which a CU runs few waves.  Results are unchanged (issue
order only).

The shipped sources are copied to a scratch directory, the loop edited there,
and the variant built from the copy into noahmp-1_amd/lib/variants/
lib_prio<K>_<P>.so, so the product's sources and hash stay untouched.

    python tools/prio_variant.py 8:2 12:2 5:1
"""
import os
import shutil
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import noahmp_pkg  # noqa: E402,F401
from noahmp_amd import build  # noqa: E402

LOOP = """      for (int iter = 2; iter <= 20; ++iter) {
        vtrips = iter;
"""
LOOP_PRIO = """      for (int iter = 2; iter <= 20; ++iter) {
        vtrips = iter;
#ifdef NMP_PRIO_ITER
        if (iter == NMP_PRIO_ITER) __builtin_amdgcn_s_setprio(NMP_PRIO_LEVEL);
#endif
"""
AFTER = """        if (iter >= 5 && fabs(dtv) <= L(0.01) && liter == 0) liter = 1;
      }
      return ok;
"""
AFTER_PRIO = """        if (iter >= 5 && fabs(dtv) <= L(0.01) && liter == 0) liter = 1;
      }
#ifdef NMP_PRIO_ITER
      __builtin_amdgcn_s_setprio(0);
#endif
      return ok;
"""


def main(specs):
    src = build.CSRC
    for spec in specs:
        k, p = (int(x) for x in spec.split(":"))
        with tempfile.TemporaryDirectory() as td:
            csrc = os.path.join(td, "csrc")
            shutil.copytree(src, csrc)
            f = os.path.join(csrc, "sflx_kernel.hip")
            text = open(f).read()
            assert text.count(LOOP) == 1 and text.count(AFTER) == 1
            text = text.replace(LOOP, LOOP_PRIO).replace(AFTER, AFTER_PRIO)
            open(f, "w").write(text)
            flags = dict(build.SOURCE_FLAGS)
            flags["sflx_kernel.hip"] = flags["sflx_kernel.hip"] + [
                f"-DNMP_PRIO_ITER={k}", f"-DNMP_PRIO_LEVEL={p}"]
            out = os.path.join(build.LIB_DIR, "variants", f"lib_prio{k}_{p}.so")
            build.CSRC = csrc
            try:
                build.build(out=out, source_flags=flags, verbose=False, force=True)
            finally:
                build.CSRC = src
            print("built", out, flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or ["8:2"])
