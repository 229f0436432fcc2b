"""Per-kernel register / spill / scratch report of the step kernel's
instantiations (hipcc -Rpass-analysis=kernel-resource-usage), compiled with the
engine's flags plus any extra ones given on the command line.

    python tools/resource_usage.py [-DNMP_WAVES_PER_EU=5 ...]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import noahmp_pkg  # noqa: E402,F401
from noahmp_amd import build  # noqa: E402

KEYS = ["VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "SGPRs Spill",
        "VGPRs Spill"]


def demangle(name):
    m = re.match(r"_ZN3nmp16sflx_step_kernelI([fd])Lb([01])ELb([01])ELi(\d+)E", name)
    if not m:
        return name
    t, r, small, os_ = m.groups()
    return f"<{'float' if t == 'f' else 'double'},R={r},SMALL={small},OS={os_}>"


def main(extra):
    src = os.path.join(build.CSRC, "sflx_kernel.hip")
    with tempfile.TemporaryDirectory() as td:
        cmd = [build.HIPCC, "-O3", "--offload-arch=gfx950", "-std=c++17", "-ffp-contract=off",
               "-mllvm", "-disable-machine-licm", "-fno-slp-vectorize", "-mllvm", "-enable-pre=false", "-I", os.path.join(ROOT, "include"), "-I", build.CSRC,
               "--offload-device-only", "-c", src, "-o", os.path.join(td, "k.o"),
               "-Rpass-analysis=kernel-resource-usage", *extra]
        out = subprocess.run(cmd, capture_output=True, text=True, check=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark:\s+(.+?): (\S+) \[-Rpass", line)
        if not m:
            continue
        key, val = m.groups()
        if key == "Function Name":
            cur = {"kernel": demangle(val)}
            rows.append(cur)
        elif cur is not None and key in KEYS:
            cur[key] = val
    print("kernel".ljust(34) + "".join(k.split(" [")[0].rjust(13) for k in KEYS))
    for r in rows:
        if r["kernel"].startswith("<"):
            print(r["kernel"].ljust(34) + "".join(str(r.get(k, "-")).rjust(13) for k in KEYS))


if __name__ == "__main__":
    main(sys.argv[1:])
