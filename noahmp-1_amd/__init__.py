"""noahmp_amd -- MI355X-native Noah-MP column engine.

Drop-in for the reference engine slot (core/module_noahmp_engine.f90) driving
the per-column noahmp_sflx time step as a HIP kernel for gfx950.  The package
directory is ``noahmp-1_amd/``; import it as ``noahmp_amd`` through
``load_package()`` in the repo-root ``noahmp_pkg.py`` helper.
"""
from . import layout  # noqa: F401

__all__ = ["layout", "cases", "timeman", "params", "engine", "lib", "build"]
