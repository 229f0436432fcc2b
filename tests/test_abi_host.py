"""C-ABI surface and host logic (no GPU compute).

- every entry point include/noahmp_engine.h declares is exported by the built
  library and bound in lib.py;
- layout.py offsets == the header enums;
- error paths that return before touching a device;
- nmp_state_from_aos maps noahmp_state_t records (core/module_noahmp_type.f90:10-42);
- time manager / synthetic case generators."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from noahmp_amd import cases, layout as L, lib as _lib, timeman

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "noahmp_engine.h")


def _header():
    with open(HEADER) as f:
        return f.read()


def _enum_values(text):
    """NAME -> value for every NMP_* enumerator (implicit increments included)."""
    out = {}
    for body in re.findall(r"enum\s*\{(.*?)\}", text, re.S):
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        nxt = 0
        for item in body.split(","):
            item = item.strip()
            if not item:
                continue
            m = re.match(r"(\w+)\s*(?:=\s*(-?\d+))?$", item)
            assert m, item
            v = int(m.group(2)) if m.group(2) is not None else nxt
            out[m.group(1)] = v
            nxt = v + 1
    return out


def test_header_functions_exported(engine_lib):
    decl = set(re.findall(r"^\s*(?:int|int64_t|void\*?|const char\*)\s*(nmp_\w+)\s*\(", _header(), re.M))
    assert decl == set(_lib.EXPORTED_SYMBOLS)
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.library_path()], capture_output=True,
                        text=True, check=True).stdout
    exported = set(re.findall(r"\bT (nmp_\w+)$", nm, re.M))
    assert decl <= exported, decl - exported
    for name in decl:
        assert getattr(engine_lib, name) is not None


def test_probe_library_is_current():
    """The test-side probe library (__graft_entry__.build(): the shipped
    sources with narrowed windows, loaded by test_midloop_domain_exit_bit_exact
    through the same bindings) is built from the current sources: it carries
    their hash and exports every header function."""
    import __graft_entry__ as g
    from noahmp_amd import build as _b
    if not os.path.exists(g.PROBE_MIDLOOP):
        pytest.skip("probe library not built (run __graft_entry__.build())")
    nm = subprocess.run(["nm", "-D", "--defined-only", g.PROBE_MIDLOOP], capture_output=True,
                        text=True, check=True).stdout
    missing = set(_lib.EXPORTED_SYMBOLS) - set(re.findall(r"\bT (nmp_\w+)$", nm, re.M))
    assert not missing, f"stale probe library, rebuild it: missing {sorted(missing)}"
    assert _b.built_hash(g.PROBE_MIDLOOP) is not None


def test_layout_matches_header():
    e = _enum_values(_header())
    for name, (off, _w) in L.STATE_OFF.items():
        assert e[f"NMP_S_{name}"] == off, name
    assert e["NMP_NSTATE"] == L.NSTATE
    for i, n in enumerate(L.STATIC_F):
        assert e[f"NMP_F_{n}"] == i
    for i, n in enumerate(L.STATIC_I):
        assert e[f"NMP_I_{n}"] == i
    for i, n in enumerate(L.FORCING):
        assert e[f"NMP_A_{n}"] == i
    for i, n in enumerate(L.LDASIN):
        assert e[f"NMP_L_{n}"] == i
    assert e["NMP_NLDASIN"] == L.NLDASIN
    for i, n in enumerate(L.DIAG_FULL):
        assert e[f"NMP_D_{n}"] == i
    for i, n in enumerate(L.DIAG_OUT):
        assert e[f"NMP_O_{n}"] == i
    assert (e["NMP_DIAG_NONE"], e["NMP_DIAG_OUT"], e["NMP_DIAG_FULL"]) == (
        L.DIAG_NONE, L.DIAG_OUT_LEVEL, L.DIAG_FULL_LEVEL)
    for k in ("ERRSW", "ERRENG", "FIRE", "HCAN", "ZLVL", "FLERCH", "OPTVEG", "STOP"):
        assert e[f"NMP_ST_{k}"] == getattr(L, f"ST_{k}")


def test_params_struct_size():
    import ref  # oracle/ref.py: the reference dump order == struct order
    assert C.sizeof(_lib.NmpParams) == 4 * (ref.NPARAM_F + ref.NPARAM_I - 1) or \
        C.sizeof(_lib.NmpParams) == 4 * (ref.NPARAM_F + ref.NPARAM_I)


def test_abi_version_and_errors(engine_lib):
    assert engine_lib.nmp_abi_version() == 8
    for code in (0, -1, -2, -3, -4, -5, -6, -99):
        assert engine_lib.nmp_strerror(code)
    assert b"year boundary" in engine_lib.nmp_strerror(-6)
    # record sizes a host checks its own layout against (no device needed)
    assert engine_lib.nmp_type_size(0) == C.sizeof(_lib.NmpParams)
    assert engine_lib.nmp_type_size(1) == C.sizeof(_lib.NmpOptions) == 48
    assert engine_lib.nmp_type_size(2) == L.sflx_args_dtype().itemsize
    assert engine_lib.nmp_type_size(3) == -1
    assert engine_lib.nmp_set_launch_variant(None, 1) == -1
    p = _lib.NmpParams()
    h = C.c_void_p()
    good = _lib.NmpOptions(*L.options_tuple(L.CASE_NML_OPTIONS))
    # validation happens before any device is touched
    bad = _lib.NmpOptions(*L.options_tuple(L.CASE_NML_OPTIONS))
    bad.opt_run = 5
    assert engine_lib.nmp_init(C.byref(p), C.byref(bad), 0, 4, C.byref(h)) == -3
    assert engine_lib.nmp_init(C.byref(p), C.byref(good), 0, 2, C.byref(h)) == -5
    assert engine_lib.nmp_init(None, C.byref(good), 0, 4, C.byref(h)) == -1
    with pytest.raises(_lib.NmpError, match="option"):
        _lib.check(-3, "nmp_init")
    zs = (C.c_float * 4)(-0.1, -0.4, -1.0, -2.0)
    assert engine_lib.nmp_step(None, 1, 1, zs, 900.0, 1.0, 366, None, None, None, None, None,
                               None, 0, None, None) == -1
    rec = np.zeros(1, L.sflx_args_dtype())
    assert engine_lib.nmp_sflx_columns(None, rec.ctypes.data, 1) == -1
    assert engine_lib.nmp_sflx_column(None, rec.ctypes.data) == -1
    # the LDASIN / LDASOUT entries reject a missing engine before any device work
    assert engine_lib.nmp_forcing_from_ldasin(None, 1, 1, None, None, None) == -1
    assert engine_lib.nmp_forcing_from_ldasin_geo(None, 1, 1, None, None, 0.0, 1.0, 0.0, None,
                                                  None) == -1
    assert engine_lib.nmp_ldasin_ingest(None, 1, 1, 1, None, None, None, None) == -1
    assert engine_lib.nmp_ldasout_grid(None, 1, 1, 1, 16, None, None, -9999.0, None, None) == -1


def test_sflx_args_layout(tmp_path):
    """struct nmp_sflx_args (include/noahmp_engine.h) has the byte layout of
    layout.sflx_args_dtype(): the 131 noahmp_sflx dummies in dummy order
    (core/module_noahmp_func.f90:66-91), 4-byte members, no padding."""
    dt = L.sflx_args_dtype()
    names = [n for n, _, _ in L.SFLX_ARGS]
    nargs = sum(1 for n in names if n not in ("out", "status")) + 58
    assert nargs == 131
    src = tmp_path / "layout.c"
    body = "\n".join(f'printf("{n} %zu\\n", offsetof(nmp_sflx_args, {n}));' for n in names)
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "noahmp_engine.h"\n'
                   'int main(void){printf("size %zu\\n", sizeof(nmp_sflx_args));' + body +
                   "return 0;}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-o", str(exe),
                    str(src)], check=True)
    got = dict(line.split() for line in subprocess.run(
        [str(exe)], capture_output=True, text=True, check=True).stdout.split("\n") if line)
    assert int(got["size"]) == dt.itemsize
    for n in names:
        assert int(got[n]) == dt.fields[n][1], n


def test_sflx_records_round_trip():
    """SoA -> nmp_sflx_args records -> SoA is the identity (host mapping only)."""
    from golden_io import load
    g = load("single_casenml_mixed.npz")
    n = 64
    r = L.sflx_records(g["state0"][:, :n], g["isnow0"][:n], g["static_f"][:, :n],
                       g["static_i"][:, :n], g["forcing"][:, :n], g["zsoil"], g["dt"],
                       g["julian"], g["yearlen"])
    st, isn, dg, status = L.soa_from_records(r)
    assert np.array_equal(st.view(np.int32), g["state0"][:, :n].astype(np.float32).view(np.int32))
    assert np.array_equal(isn, g["isnow0"][:n])
    assert (r["lutyp"] == g["static_i"][0, :n]).all() and (r["isc"] == g["static_i"][3, :n]).all()
    assert (r["cosz"] == g["forcing"][L.FORCING.index("COSZ"), :n]).all()
    act = np.arange(3)[None, :] >= (r["isnow"][:, None] + 3)
    assert (r["ficeold"][~act] == 0).all() and (r["ficeold"][act] > 0).all()


def test_state_from_aos(engine_lib):
    """168-B noahmp_state_t records -> SoA state (SURVEY 8b mapping table)."""
    n = 3
    rec = np.zeros((n, 42), np.float32)
    ints = rec.view(np.int32)
    rec[:, 3:7] = [-0.1, -0.4, -1.0, -2.0]             # zsoil
    rec[:, 10] = [0, 1, 2]                             # nsnow (real, +)
    ints[:, 11] = [7, 10, 2]                           # lutyp
    ints[:, 12] = [6, 3, 9]                            # sltyp
    rec[:, 13], rec[:, 14] = 2.0, 0.5                  # lai, sai
    rec[:, 16:19] = [280.0, 0.1, 0.0]                  # cantmp, canwat, cansno
    rec[1, 7:10] = [0.0, 0.0, 0.05]                    # one layer: top at +0.05
    rec[2, 7:10] = [0.0, 0.30, 0.12]                   # two layers: tops +0.30, +0.12
    rec[:, 19:22] = 270.0
    rec[:, 22:25] = 1.0
    rec[:, 25:28] = 10.0
    rec[:, 28:32] = [285, 284, 283, 282]
    rec[:, 32:36] = 0.2
    rec[:, 36:40] = 0.05
    rec[:, 40] = 4900.0
    rec[:, 41] = -2.5                                  # zwt, +up
    st = np.full((L.NSTATE, n), -1.0, np.float32)
    isn = np.zeros(n, np.int32)
    si = np.zeros((L.NSTATIC_I, n), np.int32)
    assert engine_lib.nmp_state_from_aos(rec.ctypes.data, n, n, st.ctypes.data, isn.ctypes.data,
                                         si.ctypes.data) == 0
    assert list(isn) == [0, -1, -2]
    assert list(si[0]) == [7, 10, 2] and list(si[1]) == [6, 3, 9]
    np.testing.assert_allclose(st[L.s("SMC")], 0.25)
    np.testing.assert_allclose(st[L.si("ZWT")], 2.5)
    np.testing.assert_allclose(st[L.si("WA")], 4900.0)
    np.testing.assert_allclose(st[L.si("TV")], 280.0)
    z = st[L.s("ZSNSO")]
    np.testing.assert_allclose(z[3:, 0], [-0.1, -0.4, -1.0, -2.0])
    np.testing.assert_allclose(z[2:, 1], [-0.05, -0.15, -0.45, -1.05, -2.05], rtol=1e-6)
    np.testing.assert_allclose(z[1:, 2], [-0.18, -0.30, -0.40, -0.70, -1.30, -2.30], rtol=1e-6)
    assert st[L.si("SNOWH"), 2] == pytest.approx(0.30)
    assert engine_lib.nmp_state_from_aos(rec.ctypes.data, n, n - 1, st.ctypes.data,
                                         isn.ctypes.data, None) == -1


def test_timeman():
    assert timeman.yearlen(2000) == 366 and timeman.yearlen(1900) == 365
    assert timeman.yearlen(2001) == 365
    lat = np.radians([40.0])
    c_noon = timeman.cosz(lat, np.array([0.0]), 172.5, 366)
    c_night = timeman.cosz(lat, np.array([0.0]), 172.0, 366)
    assert c_noon[0] > 0.9 and c_night[0] < 0
    # cosz is solar_terms' factors combined in one fixed order (the device's
    # nmp_forcing_from_ldasin_geo takes the same factors): restated, bit for bit
    import math
    rng = np.random.default_rng(4)
    la, lo = np.radians(rng.uniform(-90, 90, 4096)), np.radians(rng.uniform(-180, 180, 4096))
    for jul in (0.0, 80.0, 172.3125, 365.9583):
        sd, cd, ha0 = timeman.solar_terms(jul, 366)
        decl = 0.409 * math.sin(2.0 * math.pi * (jul - 80.0) / 366)
        assert (sd, cd) == (math.sin(decl), math.cos(decl))
        assert ha0 == 2.0 * math.pi * (((jul - math.floor(jul)) * 24.0) / 24.0)
        want = np.sin(la) * sd + (np.cos(la) * cd) * np.cos((ha0 + lo) - math.pi)
        assert np.array_equal(timeman.cosz(la, lo, jul, 366).view(np.int64), want.view(np.int64))


@pytest.mark.parametrize("kind", ["casenml", "mixed", "conus"])
def test_case_generator_consistency(ref_params, kind):
    cols = cases.make_columns(512 if kind != "casenml" else 4, kind, ref_params, seed=3)
    isn = cols.isnow
    assert ((isn >= -3) & (isn <= 0)).all()
    snl = cols.state[L.s("SNICE")]
    for k in range(3):
        act = (k - 2) >= isn + 1
        assert (snl[k, act] > 0).all() and (snl[k, ~act] == 0).all()
    z = cols.state[L.s("ZSNSO")]
    assert (np.diff(z, axis=0)[np.isfinite(np.diff(z, axis=0))] <= 0).sum() > 0
    smc = cols.state[L.s("SMC")]
    sh2o = cols.state[L.s("SH2O")]
    assert (sh2o <= smc + 1e-7).all()
    f = cases.forcing_step(cols, 180.0, 366, 0, seed=1)
    assert f.shape == (L.NFORCING, cols.n) and np.isfinite(f).all()


def test_kernel_emits_every_output_once():
    """Static check of csrc/sflx_kernel.hip: every NMP_D_* diagnostic is emitted
    exactly once through the output sink and every state field is stored."""
    from collections import Counter
    src = open(os.path.join(ROOT, "noahmp-1_amd", "csrc", "sflx_kernel.hip")).read()
    c = Counter(re.findall(r"d<NMP_D_(\w+)>", src))
    assert {d for d in L.DIAG_FULL if c[d] != 1} == set(), c
    stored = set(re.findall(r"out\.s\(NMP_S_(\w+)", src)) | set(
        re.findall(r"so\[\(?NMP_S_(\w+)", src))
    assert {n for n, _ in L.STATE_FIELDS} <= stored


def test_library_carries_its_source_hash(engine_lib):
    """Build provenance: the library reports the hash of the sources it was
    compiled from, and it is the hash of the sources in this tree."""
    from noahmp_amd import build
    assert engine_lib.nmp_build_hash().decode() == build.source_hash()
    assert build.built_hash() == build.source_hash()


def test_stale_library_is_refused(tmp_path, monkeypatch):
    """A library whose embedded hash differs from the sources is refused by
    lib.load() (no silent run of a stale kernel)."""
    import importlib
    from noahmp_amd import build
    lib_mod = importlib.import_module("noahmp_amd.lib")
    stale = tmp_path / "libnoahmp_engine.so"
    data = open(build.DEFAULT_LIB_PATH, "rb").read()
    i = data.find(b"NMP_BUILD_HASH=") + 15
    stale.write_bytes(data[:i] + b"0123456789abcdef" + data[i + 16:])
    assert build.built_hash(str(stale)) == "0123456789abcdef"
    monkeypatch.setattr(build, "LIB_PATH", str(stale))
    monkeypatch.setattr(build, "DEFAULT_LIB_PATH", str(stale))
    monkeypatch.setattr(lib_mod, "_lib", None)
    with pytest.raises(RuntimeError, match="stale"):
        lib_mod.load()


def test_kernarg_layout_check():
    """The fp32 step kernels read their array bases from the kernel-argument
    segment at KArgs' byte offset 8 (sflx_kernel.hip kargs_seg); build.py
    refuses a build whose code-object metadata places it elsewhere."""
    from noahmp_amd import build

    def meta(off2):
        return ("  - .args:\n      - .offset: 0\n        .size: 8\n"
                f"      - .offset: {off2}\n        .size: 240\n        .value_kind: by_value\n"
                "    .group_segment_fixed_size: 40352\n"
                "    .name: _ZN3nmp16sflx_step_kernelIfLb1ELb0ELi1ELi0EEEvPKNS_9DevParamsENS_5KArgsIT_EE\n"
                "  - .args:\n      - .offset: 0\n"
                "    .name: _ZN3nmp20forcing_synth_kernelIfEEvllPKT_dimllPS1_\n")
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        good, bad = os.path.join(td, "good.s"), os.path.join(td, "bad.s")
        open(good, "w").write(meta(8))
        open(bad, "w").write(meta(16))
        build.check_kernarg_layout([good])
        with pytest.raises(RuntimeError, match="KArgs not at byte offset 8"):
            build.check_kernarg_layout([bad])
