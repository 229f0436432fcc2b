"""Offline run configuration: counterpart of offline/noahmp_config.py.

`Config(cfgfile)` reads the ``&NOAHMP_OFFLINE`` namelist group exactly like
the reference (offline/noahmp_config.py:47-103): the same 31 mandatory fields
(`NML_FIELDS`, :8-43), the same attribute names and the same error behaviour
(message + exit status 1).  It uses our own namelist reader (namelist.py)
instead of f90nml.

On top of the reference it maps the namelist options onto the engine's 12
`noahmp_set_options` options (core/module_noahmp_global.f90:77-112).  The
namelist has opt_tub/opt_can, which the physics does not have, and lacks
opt_crs/opt_sfc/opt_frz/opt_alb/opt_stc: those five take the
defaults suggested in global.f90 (:24,41,45,60,73) unless the namelist sets
them, and opt_tub/opt_can are carried but unused.
"""
from __future__ import annotations

import datetime
import os
import re
import sys

from . import layout as L
from . import namelist

NML_FIELDS = ["static_parameter_file", "initialization_file", "restart_file",
              "input_directory", "input_frequency", "output_directory", "output_frequency",
              "restart_directory", "restart_frequency",
              "start_year", "start_month", "start_day", "start_hour", "start_minute",
              "start_second",
              "end_year", "end_month", "end_day", "end_hour", "end_minute", "end_second",
              "interval_seconds",
              "opt_veg", "opt_run", "opt_btr", "opt_rad", "opt_tub", "opt_can", "opt_inf",
              "opt_snf", "opt_tbot"]

# defaults for the physics options the namelist does not carry (global.f90)
MISSING_OPTION_DEFAULTS = dict(opt_crs=1, opt_sfc=1, opt_frz=1, opt_alb=2, opt_stc=1)


def _err(msg: str):
    print(msg)
    sys.exit(1)


def parse_frequency(text) -> datetime.timedelta | str:
    """'1 hour' / '3 hour' / '30 minute' / '900 second' / '1 day' -> timedelta;
    month-based frequencies ('1 month') are returned as 'Nmonth' (calendar step)."""
    if isinstance(text, (int, float)):
        return datetime.timedelta(seconds=float(text))
    m = re.fullmatch(r"\s*(\d+)\s*([A-Za-z]+?)s?\s*", str(text))
    if not m:
        raise ValueError(f"unrecognised frequency {text!r}")
    n, unit = int(m.group(1)), m.group(2).lower()
    if unit in ("month", "mon"):
        return f"{n}month"
    if unit in ("year", "yr"):
        return f"{12 * n}month"
    secs = {"second": 1, "sec": 1, "s": 1, "minute": 60, "min": 60, "hour": 3600, "hr": 3600,
            "h": 3600, "day": 86400, "d": 86400}.get(unit)
    if secs is None:
        raise ValueError(f"unrecognised frequency unit in {text!r}")
    return datetime.timedelta(seconds=n * secs)


class Config(object):
    def __init__(self, cfgfile):
        self.indir = "."
        self.infreq = None
        self.outdir = "."
        self.outfreq = None
        self.resdir = "."
        self.resfreq = None

        self.constfile = "domain.nc"
        self.initfile = "init.nc"

        self.datetimebeg = None
        self.datetimeend = None
        self.timestep = 0

        self.parse_cfg(cfgfile)

    def parse_cfg(self, cfgfile):
        if not os.path.isfile(cfgfile):
            _err(f"ERR: Unable to find configuration file {cfgfile}")
        nml = namelist.read(cfgfile)
        if "noahmp_offline" not in nml:
            _err(f"ERR: Unable to find NOAHMP_OFFLINE in configuration file {cfgfile}")
        cfg = nml["noahmp_offline"]
        for var in NML_FIELDS:
            if var not in cfg:
                _err("ERR: Unable to find {:s} in configuration file {:s}".format(var, cfgfile))
        self.raw = cfg
        # Initialization
        self.constfile = cfg["static_parameter_file"]
        self.initfile = cfg["initialization_file"]
        self.resfile = cfg["restart_file"]
        # Input & Output
        self.indir = cfg["input_directory"]
        self.infreq = cfg["input_frequency"]
        self.outdir = cfg["output_directory"]
        self.outfreq = cfg["output_frequency"]
        self.resdir = cfg["restart_directory"]
        self.resfreq = cfg["restart_frequency"]
        # Physics
        self.opt_veg = cfg["opt_veg"]
        self.opt_run = cfg["opt_run"]
        self.opt_btr = cfg["opt_btr"]
        self.opt_rad = cfg["opt_rad"]
        self.opt_inf = cfg["opt_inf"]
        self.opt_snf = cfg["opt_snf"]
        self.opt_tub = cfg["opt_tub"]
        self.opt_can = cfg["opt_can"]
        self.opt_tbot = cfg["opt_tbot"]
        # Model Temporal settings
        self.timestep = datetime.timedelta(seconds=cfg["interval_seconds"])
        self.begdatetime = datetime.datetime(cfg["start_year"], cfg["start_month"],
                                             cfg["start_day"], cfg["start_hour"],
                                             cfg["start_minute"], cfg["start_second"])
        self.enddatetime = datetime.datetime(cfg["end_year"], cfg["end_month"], cfg["end_day"],
                                             cfg["end_hour"], cfg["end_minute"],
                                             cfg["end_second"])

    # ---- additions for the engine --------------------------------------------
    def engine_options(self) -> dict:
        """The 12 noahmp_set_options values (namelist + H10 defaults)."""
        opts = {k: int(getattr(self, k)) for k in ("opt_veg", "opt_run", "opt_btr", "opt_rad",
                                                    "opt_inf", "opt_snf", "opt_tbot")}
        for k, v in MISSING_OPTION_DEFAULTS.items():
            opts[k] = int(self.raw.get(k, v))
        for k, (lo, hi) in L.OPTION_RANGES.items():
            if not lo <= opts[k] <= hi:
                _err(f"ERR: {k} = {opts[k]} outside {lo}..{hi}")
        return {k: opts[k] for k in L.OPTION_NAMES}

    def step_count(self) -> int:
        return int(round((self.enddatetime - self.begdatetime) / self.timestep))

    def step_times(self):
        """Model time at the END of each step (begdatetime + k*timestep, k = 1..n)."""
        return [self.begdatetime + (k + 1) * self.timestep for k in range(self.step_count())]

    @property
    def output_interval(self):
        return parse_frequency(self.outfreq)

    @property
    def restart_interval(self):
        return parse_frequency(self.resfreq)

    @property
    def input_interval(self):
        return parse_frequency(self.infreq)
