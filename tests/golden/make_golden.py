"""Generate the golden fixtures in tests/golden/ from the REFERENCE Fortran.

The reference ships no tests or golden vectors, so every
fixture here is produced by running the reference noahmp_sflx itself
(/root/reference/core/*.f90 compiled by oracle/Makefile into
oracle/_ref/libnoahmp_ref.so) on seeded synthetic inputs from
noahmp_amd.cases.  Each .npz holds inputs AND the reference outputs.

  params_ref_<VEG>_<SOIL>.npz   every table value as read by the reference readers
  single_<name>.npz             one noahmp_sflx call over a stratified column set
                                (single_fatal: extreme-SOLDN columns that hit wrf_error_fatal)
  traj_casenml.npz              96 steps (run/case.nml length, dt=900 s) of the
                                case.nml column + 31 mixed columns, every step
  traj_snow.npz                 480 steps (dt=1800 s) of 24 snow columns
  single_combo_*.npz            several non-default options at once (hand-picked and seeded)
  single_tbl_<name>.npz         the other parameter tables (MODIS/IGBP veg, STAS-RUC soil);
                                the fixture records its `soil`/`veg` table tags
  traj_combo_a.npz              48 steps (dt=1800 s) of 32 columns under combo_a
                                (dynamic vegetation + carbon, Chen97 surface layer, ...)
  ficeold_snow.npz              one call over melting snow columns with a caller FICEOLD
                                that differs from the step-start ice fraction (compact's
                                DDZ3, func.f90:5655)

usage (this container only; needs /root/reference):
  make -C oracle ref && python tests/golden/make_golden.py [group ...]
  groups: params single variants traj combos tables ficeold (default: all)
"""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import noahmp_pkg  # noqa: E402,F401
import ref  # noqa: E402
from noahmp_amd import cases  # noqa: E402
from noahmp_amd import layout as L  # noqa: E402

BASE = L.options_tuple(L.CASE_NML_OPTIONS)
# one fixture per non-default value of every option (global.f90:17-74)
VARIANTS = {
    "veg2": dict(opt_veg=2), "veg3": dict(opt_veg=3), "veg4": dict(opt_veg=4),
    "veg5": dict(opt_veg=5), "crs2": dict(opt_crs=2), "btr2": dict(opt_btr=2),
    "btr3": dict(opt_btr=3), "run2": dict(opt_run=2), "run3": dict(opt_run=3),
    "run4": dict(opt_run=4), "sfc2": dict(opt_sfc=2), "frz2": dict(opt_frz=2),
    "inf2": dict(opt_inf=2), "rad2": dict(opt_rad=2), "rad3": dict(opt_rad=3),
    "alb1": dict(opt_alb=1), "snf2": dict(opt_snf=2), "snf3": dict(opt_snf=3),
    "tbot2": dict(opt_tbot=2), "stc2": dict(opt_stc=2),
}
# several non-default options in one configuration (interactions between options)
COMBOS = {
    "combo_a": dict(opt_veg=2, opt_crs=2, opt_btr=2, opt_run=3, opt_sfc=2, opt_frz=2, opt_inf=2,
                    opt_rad=1, opt_alb=1, opt_snf=2, opt_tbot=2, opt_stc=2),
    "combo_b": dict(opt_veg=5, opt_btr=3, opt_run=2, opt_rad=3, opt_snf=3),
    "combo_c": dict(opt_veg=4, opt_run=4, opt_rad=2, opt_sfc=2, opt_stc=2, opt_frz=2),
}
OPTION_VALUES = dict(opt_veg=5, opt_crs=2, opt_btr=3, opt_run=4, opt_sfc=2, opt_frz=2, opt_inf=2,
                     opt_rad=3, opt_alb=2, opt_snf=3, opt_tbot=2, opt_stc=2)
# (name, soil tag, veg tag) for single calls with the other shipped tables
TABLE_CASES = [("modis", "STAS", "MODIFIED_IGBP_MODIS_NOAH"), ("ruc", "STAS-RUC", "USGS"),
               ("modis_ruc", "STAS-RUC", "MODIFIED_IGBP_MODIS_NOAH")]
TAGS = [("STAS", "USGS"), ("STAS-RUC", "USGS"), ("STAS", "MODIFIED_IGBP_MODIS_NOAH"),
        ("STAS-RUC", "MODIFIED_IGBP_MODIS_NOAH")]


def opts_with(**kw):
    d = dict(L.CASE_NML_OPTIONS)
    d.update(kw)
    return L.options_tuple(d)


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print("wrote", path, os.path.getsize(path) // 1024, "KB")


def random_combo(seed):
    rng = np.random.default_rng(seed)
    return {k: int(rng.integers(1, v + 1)) for k, v in OPTION_VALUES.items()}


def single(name, P, kind, n, seed, options, dt=1800.0, julian=180.3, yearlen=366, soldn=None,
           tags=("STAS", "USGS")):
    cols = cases.make_columns(n, kind, P, seed=seed, julian=julian)
    f = cases.forcing_random(cols, seed=seed)
    if soldn is not None:  # extreme shortwave -> ERRSW / ERRENG / FIRE fatal-status columns
        f[L.FORCING.index("SOLDN")] = np.random.default_rng(seed).uniform(*soldn, n)
    ref.configure(options, *tags)
    st, isn, dg, status = ref.step(cases.CASE_NML_ZSOIL, dt, yearlen, julian, cols.state,
                                   cols.isnow, cols.static_f, cols.static_i, f)
    save(f"single_{name}.npz", options=np.array(options, np.int32), dt=np.float32(dt),
         soil=np.array(tags[0]), veg=np.array(tags[1]),
         julian=np.float32(julian), yearlen=np.int32(yearlen), zsoil=cases.CASE_NML_ZSOIL,
         state0=cols.state, isnow0=cols.isnow, static_f=cols.static_f, static_i=cols.static_i,
         forcing=f, state1=st, isnow1=isn, diag=dg, status=status)


def trajectory(name, P, cols, nsteps, dt, julian0, yearlen, seed, options, keep_every=1):
    ref.configure(options)
    st, isn = cols.state.copy(), cols.isnow.copy()
    F, S, I, D, ST = [], [], [], [], []
    for s in range(nsteps):
        jul = julian0 + s * dt / 86400.0
        f = cases.forcing_step(cols, jul, yearlen, s, seed=seed)
        st, isn, dg, status = ref.step(cases.CASE_NML_ZSOIL, dt, yearlen, jul, st, isn,
                                       cols.static_f, cols.static_i, f)
        F.append(f)
        if (s + 1) % keep_every == 0 or s == nsteps - 1:
            S.append(st)
            I.append(isn)
            D.append(dg)
            ST.append(status)
    save(f"traj_{name}.npz", options=np.array(options, np.int32), dt=np.float32(dt),
         julian0=np.float32(julian0), yearlen=np.int32(yearlen), zsoil=cases.CASE_NML_ZSOIL,
         keep_every=np.int32(keep_every), state0=cols.state, isnow0=cols.isnow,
         static_f=cols.static_f, static_i=cols.static_i, forcing=np.stack(F),
         states=np.stack(S), isnows=np.stack(I), diags=np.stack(D), statuses=np.stack(ST))


def table_child(name, soil, veg, seed):
    ref.configure(BASE, soil, veg)
    single(f"tbl_{name}", ref.dump_params(), "conus", 512, seed, BASE, tags=(soil, veg))


def dump_params_child(soil, veg):
    ref.configure(BASE, soil, veg)
    d = ref.dump_params()
    save(f"params_ref_{veg}_{soil}.npz", **{k: np.asarray(v) for k, v in d.items()})


if __name__ == "__main__":
    if len(sys.argv) == 4 and sys.argv[1] == "--params":
        dump_params_child(sys.argv[2], sys.argv[3])
        sys.exit(0)
    if len(sys.argv) == 6 and sys.argv[1] == "--table":
        table_child(sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5]))
        sys.exit(0)
    groups = set(sys.argv[1:]) or {"params", "single", "variants", "traj", "combos", "tables",
                                    "ficeold"}
    # the reference keeps tables in process-global module arrays: one process per tag pair
    if "params" in groups:
        for soil, veg in TAGS:
            subprocess.run([sys.executable, __file__, "--params", soil, veg], check=True)
    ref.configure(BASE)
    P = ref.dump_params()
    if "single" in groups:
        single("casenml_mixed", P, "mixed", 2048, 11, BASE)
        single("casenml_conus", P, "conus", 2048, 12, BASE)
        single("fatal", P, "conus", 256, 13, BASE, soldn=(0.0, 2.0e5))
    if "variants" in groups:
        for i, (name, kw) in enumerate(VARIANTS.items()):
            single(name, P, "conus", 256, 100 + i, opts_with(**kw))
    if "traj" in groups:
        # 96-step case.nml trajectory (interval_seconds = 900, 2000-01-01 .. 01-02)
        c1 = cases.make_columns(1, "casenml", P, seed=0, julian=0.0)
        c2 = cases.make_columns(31, "mixed", P, seed=21, julian=0.0)
        cols = cases.ColumnSet(*[np.concatenate([a, b], axis=-1) for a, b in zip(
            (c1.static_f, c1.static_i, c1.state, c1.isnow, c1.lon, c1.t0, c1.amp, c1.rh, c1.pres,
             c1.wind, c1.wet),
            (c2.static_f, c2.static_i, c2.state, c2.isnow, c2.lon, c2.t0, c2.amp, c2.rh, c2.pres,
             c2.wind, c2.wet))])
        trajectory("casenml", P, cols, 96, 900.0, 0.0, 366, 5, BASE)
        snow = cases.make_columns(400, "conus", P, seed=33, julian=15.0)
        pick = np.nonzero(snow.isnow < 0)[0][:24]
        trajectory("snow", P, snow.take(pick), 480, 1800.0, 15.0, 366, 7, BASE, keep_every=8)
    if "combos" in groups:
        for i, (name, kw) in enumerate(COMBOS.items()):
            single(name, P, "conus", 512, 200 + i, opts_with(**kw))
        for i in range(3):
            single(f"combo_r{i}", P, "conus", 512, 300 + i, opts_with(**random_combo(300 + i)))
        cols = cases.make_columns(32, "conus", P, seed=41, julian=120.0)
        trajectory("combo_a", P, cols, 48, 1800.0, 120.0, 366, 9, opts_with(**COMBOS["combo_a"]))
    if "tables" in groups:
        for i, (name, soil, veg) in enumerate(TABLE_CASES):
            subprocess.run([sys.executable, __file__, "--table", name, soil, veg, str(400 + i)],
                           check=True)
    if "ficeold" in groups:
        # warm steps over snow columns, so layers melt (IMELT = 1) and compaction
        # reads FICEOLD; the caller's FICEOLD is the step-start fraction scaled
        # up towards 1 (ice fraction at the previous step, before this melt)
        ref.configure(BASE)
        cols = cases.make_columns(2048, "mixed", P, seed=51, julian=100.0)
        pick = np.nonzero(cols.isnow < 0)[0][:512]
        cols = cols.take(pick)
        cols = cases.ColumnSet(*(np.ascontiguousarray(a) for a in (
            cols.static_f, cols.static_i, cols.state, cols.isnow, cols.lon, cols.t0, cols.amp,
            cols.rh, cols.pres, cols.wind, cols.wet)))
        f = cases.forcing_random(cols, seed=51)
        f[L.FORCING.index("SFCTMP")] = np.float32(276.0) + np.random.default_rng(52).uniform(
            0.0, 8.0, cols.n).astype(np.float32)
        sn_i = cols.state[L.s("SNICE")]
        sn_l = cols.state[L.s("SNLIQ")]
        act = np.arange(3)[:, None] >= cols.isnow[None, :] + 3
        frac = np.where(act, sn_i / np.where(act, sn_i + sn_l, 1.0), 0.0)
        w = np.random.default_rng(53).uniform(0.0, 1.0, frac.shape)
        fice = np.where(act, frac + w * (1.0 - frac), 0.0).astype(np.float32)
        st, isn, dg, status = ref.step(cases.CASE_NML_ZSOIL, 1800.0, 366, 100.3, cols.state,
                                       cols.isnow, cols.static_f, cols.static_i, f, ficeold=fice)
        save("ficeold_snow.npz", options=np.array(BASE, np.int32), dt=np.float32(1800.0),
             julian=np.float32(100.3), yearlen=np.int32(366), zsoil=cases.CASE_NML_ZSOIL,
             state0=cols.state, isnow0=cols.isnow, static_f=cols.static_f,
             static_i=cols.static_i, forcing=f, ficeold=fice, state1=st, isnow1=isn, diag=dg,
             status=status)
