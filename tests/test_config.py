"""Host side of the offline path: namelist reader, Config (counterpart of
offline/noahmp_config.py), frequencies, output/restart boundaries."""
import datetime

import pytest

from noahmp_amd import config, driver, namelist

CASE = """&NOAHMP_OFFLINE
  static_parameter_file = 'geo_em.d01.nc'   ! trailing comment
  initialization_file = "init.nc"
  restart_file = 'restart.nc'
  input_directory = 'ldasin'
  input_frequency = '1 hour'
  output_directory = '{out}'
  output_frequency = '3 hour'
  restart_directory = '{res}'
  restart_frequency = '1 month'
  start_year = 2000, start_month = 1, start_day = 1
  start_hour = 0  start_minute = 0  start_second = 0
  end_year = 2000 end_month = 1 end_day = 2 end_hour = 0 end_minute = 0 end_second = 0
  interval_seconds = 900
  opt_veg = 1, opt_run = 1, opt_btr = 1, opt_rad = 1, opt_tub = 1, opt_can = 1
  opt_inf = 1, opt_tbot = 1, opt_snf = 1
/
"""


def write_case(tmp_path, **extra):
    text = CASE.format(out=tmp_path / "out", res=tmp_path / "res")
    if extra:
        text = text.replace("/\n", "".join(f"  {k} = {v}\n" for k, v in extra.items()) + "/\n")
    p = tmp_path / "case.nml"
    p.write_text(text)
    return str(p)


def test_namelist_values():
    g = namelist.reads("&grp a = 1, b=2.5d0 c = 'x''y', d = .true., e = 3*0.5, 1 / junk &g2 z=-1e-3 /")
    assert g["grp"] == {"a": 1, "b": 2.5, "c": "x'y", "d": True, "e": [0.5, 0.5, 0.5, 1]}
    assert g["g2"]["z"] == -1e-3
    with pytest.raises(namelist.NamelistError):
        namelist.reads("&grp a = 1")


def test_config_matches_reference_semantics(tmp_path):
    c = config.Config(write_case(tmp_path))
    # the attribute set the reference Config exposes (SURVEY.md 8f / offline/noahmp_config.py)
    for attr in ("begdatetime", "constfile", "datetimebeg", "datetimeend", "enddatetime", "indir",
                 "infreq", "initfile", "opt_btr", "opt_can", "opt_inf", "opt_rad", "opt_run",
                 "opt_snf", "opt_tbot", "opt_tub", "opt_veg", "outdir", "outfreq", "resdir",
                 "resfile", "resfreq", "timestep"):
        assert hasattr(c, attr), attr
    assert c.timestep == datetime.timedelta(seconds=900)
    assert c.step_count() == 96
    assert c.begdatetime == datetime.datetime(2000, 1, 1)
    assert c.output_interval == datetime.timedelta(hours=3)
    assert c.restart_interval == "1month"
    opts = c.engine_options()
    assert opts == {"opt_veg": 1, "opt_crs": 1, "opt_btr": 1, "opt_run": 1, "opt_sfc": 1,
                    "opt_frz": 1, "opt_inf": 1, "opt_rad": 1, "opt_alb": 2, "opt_snf": 1,
                    "opt_tbot": 1, "opt_stc": 1}
    c2 = config.Config(write_case(tmp_path, opt_sfc=2, opt_alb=1))
    assert c2.engine_options()["opt_sfc"] == 2 and c2.engine_options()["opt_alb"] == 1


def test_config_errors(tmp_path, capsys):
    with pytest.raises(SystemExit) as e:
        config.Config(str(tmp_path / "missing.nml"))
    assert e.value.code == 1 and "Unable to find configuration file" in capsys.readouterr().out
    p = tmp_path / "bad.nml"
    p.write_text(CASE.format(out="o", res="r").replace("  interval_seconds = 900\n", ""))
    with pytest.raises(SystemExit):
        config.Config(str(p))
    assert "Unable to find interval_seconds" in capsys.readouterr().out
    with pytest.raises(SystemExit):
        config.Config(write_case(tmp_path, opt_run=7)).engine_options()


def test_frequencies_and_boundaries():
    assert config.parse_frequency("30 minutes") == datetime.timedelta(minutes=30)
    assert config.parse_frequency("1 day") == datetime.timedelta(days=1)
    assert config.parse_frequency("2 years") == "24month"
    t0 = datetime.datetime(2000, 1, 1)
    every = datetime.timedelta(hours=3)
    hits = [k for k in range(1, 97)
            if driver._is_boundary(t0 + k * datetime.timedelta(seconds=900), t0, every)]
    assert hits == [12 * i for i in range(1, 9)]  # 8 outputs in one day at 3-hourly
    assert driver._is_boundary(datetime.datetime(2000, 2, 1), t0, "1month")
    assert not driver._is_boundary(datetime.datetime(2000, 2, 1, 0, 15), t0, "1month")
    assert not driver._is_boundary(t0, t0, "1month")


def test_coherent_order_is_a_permutation_grouping_keys():
    """order.coherent_order: a permutation; within a longitude band the
    snow-free and snow-covered columns, and the vegetation types, are grouped."""
    import numpy as np
    from noahmp_amd import cases, layout as L
    from noahmp_amd.order import KEYS, coherent_order
    from noahmp_amd.params import Params
    cols = cases.make_columns(5000, "mixed", Params.builtin().as_dict(), seed=8)
    for key in KEYS:
        p = coherent_order(cols.lon, cols.static_i, cols.isnow, key)
        assert np.array_equal(np.sort(p), np.arange(5000))
    p = coherent_order(cols.lon, cols.static_i, cols.isnow, "lon-snow-type", band_deg=4.0)
    band = np.floor(np.degrees(cols.lon[p]) / 4.0)
    assert (np.diff(band) >= 0).all()
    snow = (cols.isnow[p] < 0).astype(int)
    vt = cols.static_i[L.STATIC_I.index("VEGTYP")][p]
    for b in np.unique(band)[:5]:
        m = band == b
        assert (np.diff(snow[m]) >= 0).all()
        for sv in (0, 1):
            assert (np.diff(vt[m][snow[m] == sv]) >= 0).all()
