"""Kubernetes resource quantities (the subset of apimachinery's resource.Quantity
that schedulers and quota controllers need), with exact rational arithmetic.

``parse("100m") == Fraction(1, 10)``, ``parse("1Gi") == 2**30``,
``milli_value("0.5") == 500``, ``value("1.2") == 2`` (Value() rounds up, like
apimachinery).
"""
from __future__ import annotations

import math
import re
from fractions import Fraction

_BIN = {"Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}
_DEC = {"n": Fraction(1, 10 ** 9), "u": Fraction(1, 10 ** 6), "m": Fraction(1, 1000), "": Fraction(1),
        "k": Fraction(10 ** 3), "M": Fraction(10 ** 6), "G": Fraction(10 ** 9), "T": Fraction(10 ** 12),
        "P": Fraction(10 ** 15), "E": Fraction(10 ** 18)}
_RE = re.compile(r"^([+-]?(?:\d+\.?\d*|\.\d+))(?:([eE][+-]?\d+)|(Ki|Mi|Gi|Ti|Pi|Ei|n|u|m|k|M|G|T|P|E))?$")

Quantity = Fraction


def parse(q) -> Fraction:
    """Parse a quantity string (or int/float/Fraction) into an exact Fraction."""
    if isinstance(q, Fraction):
        return q
    if isinstance(q, bool):
        raise ValueError("bool is not a quantity")
    if isinstance(q, int):
        return Fraction(q)
    if isinstance(q, float):
        return Fraction(q).limit_denominator(10 ** 9)
    s = str(q).strip()
    m = _RE.match(s)
    if not m:
        raise ValueError(f"invalid quantity {q!r}")
    num, exp, suf = m.groups()
    v = Fraction(num)
    if exp:
        v *= Fraction(10) ** int(exp[1:])
    elif suf:
        v *= _BIN[suf] if suf in _BIN else _DEC[suf]
    return v


def value(q) -> int:
    """Integer value rounded up (apimachinery Quantity.Value())."""
    return math.ceil(parse(q))


def milli_value(q) -> int:
    """Milli-units rounded up (Quantity.MilliValue())."""
    return math.ceil(parse(q) * 1000)


def fmt(v, binary: bool = False) -> str:
    """Canonical-ish string form (integers stay integers, fractions use m)."""
    v = parse(v)
    if v.denominator == 1:
        iv = int(v)
        if binary and iv and iv % 2 ** 30 == 0:
            return f"{iv // 2 ** 30}Gi"
        if binary and iv and iv % 2 ** 20 == 0:
            return f"{iv // 2 ** 20}Mi"
        return str(iv)
    mv = v * 1000
    if mv.denominator == 1:
        return f"{int(mv)}m"
    return str(float(v))


def from_milli(m: int) -> Fraction:
    return Fraction(m, 1000)


# -------------------------------------------------- ResourceList helpers
def rl_parse(rl: dict | None) -> dict[str, Fraction]:
    return {k: parse(v) for k, v in (rl or {}).items()}


def rl_add(a: dict, b: dict) -> dict[str, Fraction]:
    """quota.Add: union of keys, values summed."""
    out = {k: parse(v) for k, v in a.items()}
    for k, v in b.items():
        out[k] = out.get(k, Fraction(0)) + parse(v)
    return out


def rl_max(a: dict, b: dict) -> dict[str, Fraction]:
    """quota.Max: union of keys, element-wise max."""
    out = {k: parse(v) for k, v in a.items()}
    for k, v in b.items():
        pv = parse(v)
        out[k] = max(out[k], pv) if k in out else pv
    return out


def rl_sub(a: dict, b: dict) -> dict[str, Fraction]:
    out = {k: parse(v) for k, v in a.items()}
    for k, v in b.items():
        out[k] = out.get(k, Fraction(0)) - parse(v)
    return out


def rl_fmt(rl: dict) -> dict[str, str]:
    return {k: fmt(v, binary=(k in ("memory", "ephemeral-storage"))) for k, v in rl.items()}


def rl_equal(a: dict, b: dict) -> bool:
    ka = {k for k, v in a.items() if parse(v) != 0}
    kb = {k for k, v in b.items() if parse(v) != 0}
    return ka == kb and all(parse(a[k]) == parse(b[k]) for k in ka)
