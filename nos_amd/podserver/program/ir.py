"""Program IR: values, nodes, limits and the op sets (shared by the
validator, the accounting, the compiler and the executor)."""
from __future__ import annotations

import math
from dataclasses import dataclass, field

FORMAT = "nos-amd.program/v1"
WIRE_DTYPES = {"fp32": 4, "bf16": 2, "i32": 4}   # i32: token ids (an input only; consumed by embedding)
FLOAT_DTYPES = ("fp32", "bf16")
MAX_NODES = 8192
MAX_PARAMS = 8192
MAX_NUMEL = 1 << 31          # elements of one value
MAX_RANK = 8
MAX_VARIANTS = 8             # input shapes one tenant may register (parse_variants)
UNARY = ("gelu", "relu", "sigmoid", "silu", "tanh", "exp", "neg", "rsqrt")
BINARY = ("add", "mul", "sub", "div")
ACTS = (None, "gelu", "relu")
INTERP_MODES = ("bicubic", "bilinear", "nearest")


class ProgramError(ValueError):
    """The program is malformed or uses something the server does not run."""


@dataclass(frozen=True)
class Value:
    name: str
    shape: tuple[int, ...]
    dtype: str
    kind: str                 # "input" | "param" | "state" | "node"

    @property
    def numel(self) -> int:
        return math.prod(self.shape)

    @property
    def nbytes(self) -> int:
        return self.numel * WIRE_DTYPES[self.dtype]


@dataclass
class Node:
    op: str
    inputs: list[str]
    output: str
    attrs: dict = field(default_factory=dict)



# ---------------------------------------------------------------- validation
def _req(cond: bool, msg: str) -> None:
    if not cond:
        raise ProgramError(msg)


def _int(v, what: str, lo: int | None = None) -> int:
    _req(isinstance(v, int) and not isinstance(v, bool), f"{what} must be an integer, got {v!r}")
    if lo is not None:
        _req(v >= lo, f"{what} must be >= {lo}, got {v}")
    return v


def _dim(d, what: str) -> int:
    """One dimension: an int in [1, MAX_NUMEL] (products are then taken on
    Python ints, which cannot wrap)."""
    d = _int(d, what, 1)
    _req(d <= MAX_NUMEL, f"{what} {d} is over {MAX_NUMEL}")
    return d


def _shape(v, what: str) -> tuple[int, ...]:
    _req(isinstance(v, list) and len(v) <= MAX_RANK, f"{what} must be a list of at most {MAX_RANK} dims")
    s = tuple(_dim(d, f"{what} dim") for d in v)
    _req(math.prod(s) <= MAX_NUMEL, f"{what} has more than {MAX_NUMEL} elements")
    return s


def _name(v, what: str) -> str:
    _req(isinstance(v, str) and 0 < len(v) <= 128, f"{what} must be a non-empty string of <= 128 chars")
    return v


def _broadcast(a: tuple, b: tuple, what: str) -> tuple:
    n = max(len(a), len(b))
    a2, b2 = (1,) * (n - len(a)) + a, (1,) * (n - len(b)) + b
    out = []
    for x, y in zip(a2, b2):
        _req(x == y or x == 1 or y == 1, f"{what}: shapes {a} and {b} do not broadcast")
        out.append(max(x, y))
    return tuple(out)




def _pair(v, what: str, lo: int) -> tuple[int, int]:
    if isinstance(v, int) and not isinstance(v, bool):
        v = [v, v]
    _req(isinstance(v, list) and len(v) == 2, f"{what} must be an int or [h, w]")
    return (_int(v[0], what, lo), _int(v[1], what, lo))


def _eps(a: dict, what: str) -> None:
    eps = a.get("eps", 1e-5)
    _req(isinstance(eps, (int, float)) and not isinstance(eps, bool) and 0 < eps < 1, f"{what}: eps must be in (0, 1)")



OPS = ("linear", "layernorm", "attention", *BINARY, *UNARY, "cat", "slice", "reshape", "permute", "expand",
       "cast", "interpolate",
       # general tenants: conv nets and decoder LLMs (nos_amd/ops/tenant.py)
       "conv2d", "batchnorm", "max_pool2d", "avg_pool2d", "mean", "sum", "matmul", "softmax", "embedding",
       "rmsnorm", "rotary", "sdpa")
# stateful decoding (round 6): ops over state buffers that persist across a
# tenant's requests (a K / V cache, a position counter).  STATE_WRITERS update
# their first input IN PLACE and return its new version (the validator makes
# the old version dead from then on, so in-place equals SSA semantics)
STATE_OPS = ("kv_write", "sdpa_cache", "rotary_at", "pos_add", "pos_set", "argmax")
STATE_WRITERS = ("kv_write", "pos_add", "pos_set")
STATE_DTYPES = ("fp32", "bf16", "i32")
MAX_STATE = 1024
OPS = OPS + STATE_OPS
NEVER_FOLD = ("attention", "sdpa", *STATE_OPS)
# step kinds that run a gfx950 kernel of libnos_hip.so (CompiledProgram.stats["kernels"])
NATIVE_KINDS = ("linear", "linear_ln", "linear_rms", "ln_qkv_attention", "attention", "layernorm", "conv2d", "matmul",
                "softmax", "embedding", "rmsnorm", "rotary", "sdpa", "patches", "unary", "kv_write", "sdpa_cache",
                "rotary_at", "pos_add", "pos_set", "argmax", "glu")
GEMM_OPS = ("linear", "conv2d")


def torch_dtype(dt: str):
    import torch

    return {"fp32": torch.float32, "bf16": torch.bfloat16, "i32": torch.int32}[dt]
