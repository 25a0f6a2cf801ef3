"""Label selectors (string form and LabelSelector objects), field selectors and
RFC 7386 JSON merge patch -- the apimachinery pieces the API server needs."""
from __future__ import annotations

import copy
import re
from typing import Any, Callable

# ------------------------------------------------------------ label selectors
_SET_RE = re.compile(r"^\s*([\w./-]+)\s+(in|notin)\s+\(([^)]*)\)\s*$")


def _split_top(s: str) -> list[str]:
    out, depth, cur = [], 0, []
    for ch in s:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            out.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    if cur:
        out.append("".join(cur))
    return [p.strip() for p in out if p.strip()]


Requirement = tuple[str, str, tuple[str, ...]]  # (key, op, values)


def parse_label_selector(s: str | None) -> list[Requirement]:
    reqs: list[Requirement] = []
    if not s:
        return reqs
    for part in _split_top(s):
        m = _SET_RE.match(part)
        if m:
            vals = tuple(v.strip() for v in m.group(3).split(",") if v.strip())
            reqs.append((m.group(1), m.group(2), vals))
        elif "!=" in part:
            k, v = part.split("!=", 1)
            reqs.append((k.strip(), "!=", (v.strip(),)))
        elif "==" in part:
            k, v = part.split("==", 1)
            reqs.append((k.strip(), "=", (v.strip(),)))
        elif "=" in part:
            k, v = part.split("=", 1)
            reqs.append((k.strip(), "=", (v.strip(),)))
        elif part.startswith("!"):
            reqs.append((part[1:].strip(), "!exists", ()))
        else:
            reqs.append((part.strip(), "exists", ()))
    return reqs


def selector_from_object(sel: dict | None) -> list[Requirement] | None:
    """metav1.LabelSelector -> requirements; None selector matches nothing, {} everything."""
    if sel is None:
        return None
    reqs: list[Requirement] = [(k, "=", (v,)) for k, v in (sel.get("matchLabels") or {}).items()]
    for e in sel.get("matchExpressions") or []:
        op = e["operator"]
        vals = tuple(e.get("values") or ())
        reqs.append((e["key"], {"In": "in", "NotIn": "notin", "Exists": "exists",
                                "DoesNotExist": "!exists"}[op], vals))
    return reqs


def match_labels(reqs: list[Requirement] | None, labels: dict[str, str]) -> bool:
    if reqs is None:
        return False
    for k, op, vals in reqs:
        has = k in labels
        v = labels.get(k)
        if op == "=" and v != vals[0]:
            return False
        if op == "!=" and has and v == vals[0]:
            return False
        if op == "in" and (not has or v not in vals):
            return False
        if op == "notin" and has and v in vals:
            return False
        if op == "exists" and not has:
            return False
        if op == "!exists" and has:
            return False
    return True


# ------------------------------------------------------------ field selectors
def _field(obj: dict, path: str) -> Any:
    cur: Any = obj
    for p in path.split("."):
        if not isinstance(cur, dict):
            return None
        cur = cur.get(p)
    return cur


def parse_field_selector(s: str | None) -> list[tuple[str, str, str]]:
    out = []
    if not s:
        return out
    for part in _split_top(s):
        if "!=" in part:
            k, v = part.split("!=", 1)
            out.append((k.strip(), "!=", v.strip()))
        else:
            k, v = part.replace("==", "=").split("=", 1)
            out.append((k.strip(), "=", v.strip()))
    return out


def match_fields(reqs: list[tuple[str, str, str]], obj: dict,
                 indexers: dict[str, Callable[[dict], Any]] | None = None) -> bool:
    for path, op, val in reqs:
        fn = (indexers or {}).get(path)
        got = fn(obj) if fn else _field(obj, path)
        got = "" if got is None else str(got)
        if (op == "=" and got != val) or (op == "!=" and got == val):
            return False
    return True


# ------------------------------------------------------------ merge patch
def merge_patch(target: Any, patch: Any) -> Any:
    """RFC 7386 JSON merge patch (returns a new object)."""
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    out = copy.deepcopy(target) if isinstance(target, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out
