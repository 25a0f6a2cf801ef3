"""Building wire programs with numpy only (the pod side never imports
torch), saving / loading them, and the GEMM-MLP probe tenant."""
from __future__ import annotations

import math

import numpy as np

from .ir import FORMAT


def bf16_bits(a: np.ndarray) -> np.ndarray:
    """float32 -> bf16 bit patterns (round to nearest even), as uint16."""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)
    r = ((u >> 16) & 1) + 0x7FFF
    return ((u + r) >> 16).astype(np.uint16)


def bf16_to_f32(bits: np.ndarray) -> np.ndarray:
    return (bits.astype(np.uint32) << 16).view(np.float32)


class Builder:
    """Assemble a wire program with numpy only (the pod side never imports
    torch).  ``param`` appends a weight to the payload; op methods append
    nodes and return the output's name."""

    def __init__(self, name: str):
        self.name = name
        self.inputs: list[dict] = []
        self.params: list[dict] = []
        self.nodes: list[dict] = []
        self.states: list[dict] = []
        self.chunks: list[bytes] = []
        self.offset = 0
        self._n = 0

    def input(self, name: str, shape, dtype: str = "fp32") -> str:
        self.inputs.append({"name": name, "shape": list(shape), "dtype": dtype})
        return name

    def param(self, name: str, array: np.ndarray, dtype: str = "fp32") -> str:
        a = np.ascontiguousarray(array, dtype=np.float32)
        raw = (a if dtype == "fp32" else bf16_bits(a)).tobytes()
        self.params.append({"name": name, "shape": list(a.shape), "dtype": dtype, "offset": self.offset,
                            "nbytes": len(raw)})
        self.chunks.append(raw)
        self.offset += len(raw)
        return name

    def state(self, name: str, shape, dtype: str = "fp32") -> str:
        """A state buffer (zero at registration, kept across requests)."""
        self.states.append({"name": name, "shape": list(shape), "dtype": dtype})
        return name

    def op(self, op: str, *inputs: str, out: str | None = None, **attrs) -> str:
        self._n += 1
        out = out or f"%{self._n}"
        self.nodes.append({"op": op, "inputs": list(inputs), "output": out,
                           "attrs": {k: v for k, v in attrs.items() if v is not None}})
        return out

    def build(self, outputs: list[str]) -> tuple[dict, bytes]:
        prog = {"format": FORMAT, "name": self.name, "inputs": self.inputs, "params": self.params,
                "nodes": self.nodes, "outputs": list(outputs)}
        if self.states:
            prog["state"] = self.states
        return prog, b"".join(self.chunks)


def save_program(prefix: str, program: dict, weights: bytes) -> None:
    """A built program as ``<prefix>.json`` + ``<prefix>.bin`` (a tenant
    builds once -- e.g. with torch.fx -- and its pods ship the files)."""
    import json

    with open(prefix + ".json", "w") as f:
        json.dump(program, f)
    with open(prefix + ".bin", "wb") as f:
        f.write(weights)


def load_program(prefix: str) -> tuple[dict, bytes]:
    """:func:`save_program`'s files back (JSON + raw bytes: nothing executable)."""
    import json

    with open(prefix + ".json") as f:
        program = json.load(f)
    with open(prefix + ".bin", "rb") as f:
        return program, f.read()


def mlp_program(dim: int = 1024, layers: int = 4, batch: int = 256, dtype: str = "bf16", seed: int = 0,
                hidden: int | None = None) -> tuple[dict, bytes]:
    """The GEMM-MLP probe tenant (BASELINE config 4's workload): ``layers``
    pre-LN residual MLP blocks (LN -> fc1 + GELU -> fc2 + residual) on a
    ``batch x dim`` activation; every block lowers onto two GEMMs with fused
    LN prologue / GELU and residual epilogues."""
    rng = np.random.default_rng(seed)
    hid = hidden or 4 * dim
    b = Builder(f"mlp-{dim}x{layers}")
    x = b.input("x", [batch, dim], "fp32")
    h = b.op("cast", x, dtype=dtype) if dtype != "fp32" else x
    for i in range(layers):
        g = b.param(f"l{i}.ln_w", 1.0 + 0.1 * rng.standard_normal(dim), dtype)
        be = b.param(f"l{i}.ln_b", 0.1 * rng.standard_normal(dim), dtype)
        w1 = b.param(f"l{i}.fc1_w", rng.standard_normal((hid, dim)) / math.sqrt(dim), dtype)
        b1 = b.param(f"l{i}.fc1_b", 0.02 * rng.standard_normal(hid), dtype)
        w2 = b.param(f"l{i}.fc2_w", rng.standard_normal((dim, hid)) / math.sqrt(hid), dtype)
        b2 = b.param(f"l{i}.fc2_b", 0.02 * rng.standard_normal(dim), dtype)
        y = b.op("layernorm", h, g, be, eps=1e-5)
        y = b.op("gelu", b.op("linear", y, w1, b1))
        h = b.op("add", b.op("linear", y, w2, b2), h)
    return b.build([h])

