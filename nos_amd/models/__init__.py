"""Tenant workloads run inside GPU slices.

Submodules load lazily: a pod-server client pod (``models.pod`` with
``NOS_AMD_POD_SERVER``) must start without importing torch.
"""
from __future__ import annotations

import importlib

_LAZY = {"YolosConfig": "yolos", "YolosDetector": "yolos", "GraphedTenant": "yolos", "make_demo_input": "yolos"}


def __getattr__(name: str):
    if name in _LAZY:
        return getattr(importlib.import_module(f".{_LAZY[name]}", __name__), name)
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
