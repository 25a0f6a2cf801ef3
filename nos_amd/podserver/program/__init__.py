"""Tenant programs: what a fractional pod ships to the pod server.

MPS runs any CUDA client program in the server's context
(``/root/reference/docs/en/docs/dynamic-gpu-partitioning/partitioning-modes-comparison.md:34-35``,
``getting-started-mps.md:22-55``).  The MI355X pod server (server.py) cannot
run foreign machine code safely in its one HIP context, so a tenant ships a
*program* instead: a static op graph over a whitelisted set of nos-amd ops
plus its weights as raw tensor bytes.  Nothing in it is executable -- no
pickle, no code -- and every op lowers onto the gfx950 kernels of
``libnos_hip.so`` (``nos_amd.ops``), so native kernels run by construction.

Wire form (JSON object; the weights travel as the message payload)::

    {"format": "nos-amd.program/v1", "name": "yolos-small",
     "inputs":  [{"name": "x", "shape": [1, 3, 800, 1066], "dtype": "fp32"}],
     "params":  [{"name": "w0", "shape": [384, 768], "dtype": "fp32", "offset": 0, "nbytes": 1179648}, ...],
     "nodes":   [{"op": "linear", "inputs": ["x", "w0", "b0"], "output": "h0", "attrs": {"act": "gelu"}}, ...],
     "outputs": ["logits", "boxes"]}

Values are SSA names; nodes are listed in execution order.  Wire dtypes are
``fp32`` (IEEE float32, little endian) and ``bf16`` (the upper 16 bits of a
float32, little-endian uint16).

:func:`parse` validates a program completely before anything is allocated:
the op whitelist, every attribute, the topological order and the exact shape
and dtype of every value (shape inference), the native kernels' constraints
on a GPU (head_dim 64, K % 64 for bf16 GEMMs, ...), the payload layout, and
an upper bound of the device bytes it needs (:attr:`Program.bytes_estimate`)
that the server checks against the tenant's slice before building.

:meth:`Program.compile` is a small graph compiler:

1. **constant folding** -- every node whose inputs are all weights runs once
   at load time on the device (e.g. YOLOS's bicubic position-embedding
   interpolation), its result becomes a weight;
2. **LayerNorm folding** -- ``layernorm -> linear`` becomes one
   ``linear_ln`` GEMM (the norm folded into the weight,
   :func:`nos_amd.ops.fold_layernorm`, statistics in the GEMM prologue);
3. **epilogue fusion** -- an activation (``gelu``/``relu``) and then a
   residual ``add`` after a GEMM go into its epilogue;
4. **QKV-attention fusion** -- ``linear_ln`` producing a fused QKV consumed
   only by ``attention`` becomes one node that, for fp32 tenants under the
   bf16x6 math, writes K/V straight into the attention's bf16 planes
   (``nos_gemm_ln_f32x6_qkv`` + ``nos_attn_fwd_f32x6_presplit_d64``);
5. **dead-value elimination and last-use release**: intermediates are
   dropped after their last consumer, so a HIP graph captured from the
   compiled program reuses their memory.

Later passes (round 4-5), each trimming launches or memory round trips (the
full order is in :class:`CompiledProgram`; ``NOS_AMD_SKIP_PASSES=name,...``
leaves the switchable ones out for A/B runs): ``add`` over ``cat``
distribution (position embeddings become the patch GEMM's residual), ViT
patch extraction as one strided im2col (``patchify``; bf16: the cast folded
in), cast + reshape / permute chains as one ``relayout``, row-slice
pushdown (YOLOS's last layer on its detection tokens only), BatchNorm
folding, parallel linears merged (Q / K / V, gate / up, the detection heads'
first layers), small linears over adjacent column slices merged into
block-diagonal GEMMs (``blockdiag``), RMSNorm folding, cast + activation as
one ``unary`` pass (``cast_unary``), rotary fused into ``sdpa``, a cat
written in place by its GEMM (``cat_buffer``), fp16-plane and LayerNorm
hand-offs between h3 kernels (``cat_stats``: layer 0's statistics from the
patch GEMM plus build-time constant rows), conv weight preparation.

The compiled program is a callable ``(x) -> tuple(outputs)``, captured into a
HIP graph by the server exactly like a built-in model.  :meth:`Program.reference`
runs the unfused graph eagerly in fp32 (the numerics reference of tests).

Modules (each new op touches them in this order):

* ``ir.py`` -- values, nodes, limits, op sets, validation helpers;
* ``validate.py`` -- per-op shape / dtype inference and :func:`parse`;
* ``graph.py`` -- :class:`Program`: memory accounting, weights as tensors;
* ``reference.py`` -- the eager fp32 semantics of every op (``_eager``);
* ``compile.py`` -- the lowering passes (:class:`compile.Lowered`);
* ``execute.py`` -- :class:`CompiledProgram`, the executor of the steps;
* ``builder.py`` -- numpy-only program building, save / load, the MLP probe.
"""
from __future__ import annotations

from .builder import Builder, bf16_bits, bf16_to_f32, load_program, mlp_program, save_program
from .compile import Lowered, _Step
from .execute import CompiledProgram, _relayout, _rows
from .graph import Program, _attn_ws, _workspace
from .ir import (ACTS, BINARY, FLOAT_DTYPES, FORMAT, GEMM_OPS, INTERP_MODES, MAX_NODES, MAX_NUMEL, MAX_PARAMS,
                 MAX_RANK, MAX_VARIANTS, NATIVE_KINDS, NEVER_FOLD, OPS, UNARY, WIRE_DTYPES, Node, ProgramError, Value,
                 _broadcast, _dim, _eps, _int, _name, _pair, _req, _shape, torch_dtype)
from .reference import _eager, _pair2, _qkv_views
from .validate import _infer, parse, parse_variants

__all__ = ["FORMAT", "Program", "CompiledProgram", "ProgramError", "Builder", "parse", "parse_variants", "mlp_program",
           "bf16_bits", "save_program", "load_program", "bf16_to_f32", "OPS", "torch_dtype", "Value", "Node",
           "Lowered"]
