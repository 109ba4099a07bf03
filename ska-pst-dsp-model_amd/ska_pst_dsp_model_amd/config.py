"""Configuration: rational oversampling factors and ``test.config.json`` sub-configs.

Mirrors ``matlab/default_config.m:12-35`` (struct with ``os_factor.nu/de``,
``n_chan``, ``fir_filter_path``, ``dtype='single'``) and
``python/data_gen/config.py:35-41`` (``load_config(sub_config_name)``).  The JSON
schema is the reference's (``config/test.config.json``); the packaged copy
(``config/test.config.json`` next to this package) adds the ``test`` sub-config the
reference's ``load_config()`` default asks for but its file lacks (config.py:71).
"""
from __future__ import annotations

import json
import os
from fractions import Fraction
from types import SimpleNamespace

__all__ = ["Rational", "as_rational", "config_dir", "load_config", "default_config"]

_HERE = os.path.dirname(os.path.abspath(__file__))
config_dir = os.path.normpath(os.path.join(_HERE, "..", "config"))
test_config_file_path = os.path.join(config_dir, "test.config.json")


class Rational:
    """``struct('nu', nu, 'de', de)`` (default_config.m:26-28), ``pfb.rational.Rational``."""

    def __init__(self, nu: int, de: int):
        self.nu = int(nu)
        self.de = int(de)
        if self.nu <= 0 or self.de <= 0:
            raise ValueError("os_factor must be positive")

    @classmethod
    def from_str(cls, s: str) -> "Rational":
        a, b = str(s).split("/")
        return cls(int(a), int(b))

    def normalize(self, n):
        """normalize.m:17 — n * de / nu."""
        return Fraction(self.de * n, self.nu)

    def multiply(self, n):
        """multiply.m:17 — n * nu / de."""
        return Fraction(self.nu * n, self.de)

    def __float__(self):
        return self.nu / self.de

    def __eq__(self, other):
        o = as_rational(other)
        return self.nu * o.de == o.nu * self.de

    def __hash__(self):
        f = Fraction(self.nu, self.de)
        return hash((f.numerator, f.denominator))

    def __str__(self):
        return f"{self.nu}/{self.de}"

    __repr__ = __str__


def as_rational(os_factor) -> Rational:
    if isinstance(os_factor, Rational):
        return os_factor
    if isinstance(os_factor, str):
        return Rational.from_str(os_factor)
    if isinstance(os_factor, dict):
        return Rational(os_factor["nu"], os_factor["de"])
    if isinstance(os_factor, (tuple, list)):
        return Rational(*os_factor)
    if hasattr(os_factor, "nu") and hasattr(os_factor, "de"):
        return Rational(os_factor.nu, os_factor.de)
    raise TypeError(f"cannot interpret os_factor {os_factor!r}")


def load_config(sub_config_name: str = "test", path: str = None) -> dict:
    """data_gen/config.py:35-41 — return one sub-config dictionary."""
    p = path or test_config_file_path
    if not os.path.exists(p):
        raise RuntimeError(f"Cannot find {os.path.basename(p)} in {os.path.dirname(p)}")
    with open(p) as f:
        cfg = json.load(f)
    return cfg[sub_config_name]


def default_config(tele: str, path: str = None) -> SimpleNamespace:
    """default_config.m:12-35 — struct with derived fields (os_factor, n_chan, paths)."""
    d = dict(load_config(tele, path))
    base = os.path.dirname(path) if path else config_dir
    d["config_dir"] = base
    d["dtype"] = "single"
    if "header_file_path" in d:
        d["header_file_path"] = os.path.join(base, d["header_file_path"])
    d["fir_filter_path"] = os.path.join(base, d["fir_filter_coeff_file_path"])
    d["os_factor"] = Rational.from_str(d["os_factor"])
    d["n_chan"] = d["channels"]
    d.setdefault("rndInput", False)
    d.setdefault("rmsInput", 0.0)
    d.setdefault("rndOutput", False)
    d.setdefault("rmsOutput", 0.0)
    return SimpleNamespace(**d)
