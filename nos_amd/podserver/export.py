"""torch.nn module -> pod-server program (``nos-amd.program/v1``).

A fractional pod of the reference runs any CUDA program against the MPS
server (``/root/reference/docs/en/docs/dynamic-gpu-partitioning/partitioning-modes-comparison.md:29-34``);
a pod-server tenant ships a program instead (program.py).  This module turns
an ordinary inference ``torch.nn.Module`` into one: :func:`export` traces it
with ``torch.fx`` (one symbolic trace, then shape propagation on an example
input for the static shapes the program needs) and maps every node onto the
program ops -- conv2d / batchnorm / pooling / linear / layernorm / the
elementwise and shape ops -- with the module's parameters and buffers as the
program's weights.  Control flow that depends on values, in-place ops and
ops outside the whitelist raise :class:`ExportError` naming the node.

Decoder LLMs from ``transformers`` have their own builder
(:mod:`nos_amd.models.llama_program`): their forward builds masks and rotary
tables dynamically, which a symbolic trace does not capture as static ops.
"""
from __future__ import annotations

import operator


from .program import Builder


class ExportError(ValueError):
    """The module uses something a pod-server program cannot express."""


def _pair(v) -> list[int]:
    return [int(v), int(v)] if isinstance(v, int) else [int(v[0]), int(v[1])]


def export(module, example, name: str = "module", dtype: str = "fp32") -> tuple[dict, bytes]:
    """(program, weights) of ``module`` (eval mode) for inputs shaped like
    ``example`` (one float tensor).  ``dtype``: the program's compute dtype
    (bf16: weights and the input are cast)."""
    import torch
    import torch.fx as fx
    import torch.nn as nn
    import torch.nn.functional as F
    from torch.fx.passes.shape_prop import ShapeProp

    module = module.eval()
    gm = fx.symbolic_trace(module)
    ShapeProp(gm).propagate(example)
    b = Builder(name)
    mods = dict(gm.named_modules())
    names: dict[str, str] = {}
    pcount = [0]

    def shape(n) -> list[int]:
        tm = n.meta.get("tensor_meta")
        if tm is None:
            raise ExportError(f"node {n.name}: no static tensor shape (not a tensor value?)")
        return [int(d) for d in tm.shape]

    def param(t, tag: str) -> str:
        pcount[0] += 1
        return b.param(f"p{pcount[0]}.{tag}", t.detach().float().cpu().numpy(), dtype)

    def ref(a) -> str:
        if isinstance(a, fx.Node):
            if a.name not in names:
                raise ExportError(f"value {a.name} is not a tensor the program defines")
            return names[a.name]
        raise ExportError(f"constant operand {a!r}: only tensors flow through a program")

    def emit(n, op, *ins, **attrs) -> None:
        names[n.name] = b.op(op, *ins, out=n.name, **attrs)

    act_mods = {nn.ReLU: "relu", nn.GELU: "gelu", nn.SiLU: "silu", nn.Sigmoid: "sigmoid", nn.Tanh: "tanh"}
    act_fns = {F.relu: "relu", torch.relu: "relu", F.gelu: "gelu", F.silu: "silu", torch.sigmoid: "sigmoid",
               F.sigmoid: "sigmoid", torch.tanh: "tanh", torch.exp: "exp", torch.rsqrt: "rsqrt"}
    bin_fns = {operator.add: "add", torch.add: "add", operator.mul: "mul", torch.mul: "mul", operator.sub: "sub",
               torch.sub: "sub", operator.truediv: "div", torch.div: "div"}
    for n in gm.graph.nodes:
        if n.op == "placeholder":
            if names:
                raise ExportError("a program takes exactly one input")
            x = b.input(n.name, shape(n), "fp32")
            names[n.name] = b.op("cast", x, dtype=dtype) if dtype != "fp32" else x
        elif n.op == "output":
            outs = n.args[0]
            outs = list(outs) if isinstance(outs, (tuple, list)) else [outs]
            return b.build([ref(o) for o in outs])
        elif n.op == "get_attr":
            t = gm
            for part in n.target.split("."):
                t = getattr(t, part)
            names[n.name] = param(t, n.target)
        elif n.op == "call_module":
            m = mods[n.target]
            x = ref(n.args[0])
            if isinstance(m, nn.Conv2d):
                if isinstance(m.padding, str) or m.padding_mode != "zeros":
                    raise ExportError(f"{n.target}: only zero-padded convolutions with explicit padding")
                ins = [x, param(m.weight, n.target + ".weight")]
                if m.bias is not None:
                    ins.append(param(m.bias, n.target + ".bias"))
                g = {"groups": int(m.groups)} if m.groups != 1 else {}
                emit(n, "conv2d", *ins, stride=_pair(m.stride), padding=_pair(m.padding), dilation=_pair(m.dilation),
                     **g)
            elif isinstance(m, nn.BatchNorm2d):
                if m.running_mean is None:
                    raise ExportError(f"{n.target}: BatchNorm without running statistics")
                g = m.weight if m.weight is not None else torch.ones_like(m.running_mean)
                be = m.bias if m.bias is not None else torch.zeros_like(m.running_mean)
                emit(n, "batchnorm", x, param(g, "bn.g"), param(be, "bn.b"), param(m.running_mean, "bn.mean"),
                     param(m.running_var, "bn.var"), eps=float(m.eps))
            elif type(m) in act_mods:
                emit(n, act_mods[type(m)], x)
            elif isinstance(m, nn.Linear):
                ins = [x, param(m.weight, n.target + ".weight")]
                if m.bias is not None:
                    ins.append(param(m.bias, n.target + ".bias"))
                emit(n, "linear", *ins)
            elif isinstance(m, nn.LayerNorm):
                if len(m.normalized_shape) != 1:
                    raise ExportError(f"{n.target}: LayerNorm over the last dim only")
                emit(n, "layernorm", x, param(m.weight, "ln.w"), param(m.bias, "ln.b"), eps=float(m.eps))
            elif isinstance(m, (nn.MaxPool2d, nn.AvgPool2d)):
                if getattr(m, "ceil_mode", False) or getattr(m, "dilation", 1) not in (1, (1, 1)):
                    raise ExportError(f"{n.target}: ceil_mode / dilated pooling is not supported")
                if isinstance(m, nn.AvgPool2d) and not m.count_include_pad:
                    raise ExportError(f"{n.target}: avg pooling must count padding")
                emit(n, "max_pool2d" if isinstance(m, nn.MaxPool2d) else "avg_pool2d", x, kernel=_pair(m.kernel_size),
                     stride=_pair(m.stride if m.stride is not None else m.kernel_size), padding=_pair(m.padding))
            elif isinstance(m, nn.AdaptiveAvgPool2d):
                if _pair(m.output_size) != [1, 1]:
                    raise ExportError(f"{n.target}: adaptive pooling to 1x1 only")
                emit(n, "mean", x, dims=[2, 3], keepdim=True)
            elif isinstance(m, nn.Flatten):
                emit(n, "reshape", x, shape=shape(n))
            elif isinstance(m, (nn.Identity, nn.Dropout)):
                names[n.name] = x
            elif isinstance(m, nn.Softmax):
                if m.dim not in (-1, len(shape(n)) - 1):
                    raise ExportError(f"{n.target}: softmax over the last dim only")
                emit(n, "softmax", x)
            else:
                raise ExportError(f"{n.target}: module {type(m).__name__} has no pod-server op")
        elif n.op == "call_function":
            f = n.target
            if f in bin_fns:
                a, c = n.args[0], n.args[1]
                if not isinstance(c, type(n)) or not isinstance(a, type(n)):
                    raise ExportError(f"{n.name}: {f.__name__} with a Python scalar (make it a buffer)")
                emit(n, bin_fns[f], ref(a), ref(c))
            elif f in act_fns:
                emit(n, act_fns[f], ref(n.args[0]))
            elif f in (torch.flatten, torch.reshape):
                emit(n, "reshape", ref(n.args[0]), shape=shape(n))
            elif f is torch.cat:
                emit(n, "cat", *[ref(a) for a in n.args[0]], dim=int(n.kwargs.get("dim", n.args[1] if len(n.args) > 1 else 0)))
            elif f in (F.softmax, torch.softmax):
                emit(n, "softmax", ref(n.args[0]))
            elif f is F.adaptive_avg_pool2d and _pair(n.args[1]) == [1, 1]:
                emit(n, "mean", ref(n.args[0]), dims=[2, 3], keepdim=True)
            elif f in (torch.matmul, operator.matmul):
                emit(n, "matmul", ref(n.args[0]), ref(n.args[1]))
            else:
                raise ExportError(f"{n.name}: function {getattr(f, '__name__', f)} has no pod-server op")
        elif n.op == "call_method":
            x = ref(n.args[0])
            if n.target in ("view", "reshape", "flatten"):
                emit(n, "reshape", x, shape=shape(n))
            elif n.target == "permute":
                dims = n.args[1:] if not isinstance(n.args[1], (list, tuple)) else n.args[1]
                emit(n, "permute", x, dims=[int(d) for d in dims])
            elif n.target == "transpose":
                r = len(shape(n))
                d0, d1 = int(n.args[1]) % r, int(n.args[2]) % r
                dims = list(range(r))
                dims[d0], dims[d1] = dims[d1], dims[d0]
                emit(n, "permute", x, dims=dims)
            elif n.target == "contiguous":
                names[n.name] = x
            elif n.target == "mean":
                dims = n.args[1] if len(n.args) > 1 else n.kwargs.get("dim")
                dims = [int(dims)] if isinstance(dims, int) else [int(d) for d in dims]
                emit(n, "mean", x, dims=dims, keepdim=bool(n.kwargs.get("keepdim", False)))
            elif n.target in ("relu", "sigmoid", "tanh", "exp"):
                emit(n, n.target, x)
            else:
                raise ExportError(f"{n.name}: method .{n.target}() has no pod-server op")
    raise ExportError("graph has no output")


__all__ = ["export", "ExportError"]
