"""The eager, unfused op semantics in PyTorch: the numerics reference of
:meth:`Program.reference` and the load-time constant folding."""
from __future__ import annotations

import os

from .ir import ProgramError, torch_dtype


def _eager(op: str, args: list, attrs: dict, ref: bool = False):
    """One unfused op in PyTorch (constant folding, and :meth:`Program.reference`)."""
    import torch
    import torch.nn.functional as F

    from ... import ops

    if op == "linear":
        y = F.linear(args[0], args[1], args[2] if len(args) > 2 else None)
        act = attrs.get("act")
        return F.gelu(y) if act == "gelu" else (F.relu(y) if act == "relu" else y)
    if op == "layernorm":
        x = args[0]
        return F.layer_norm(x, (x.shape[-1],), args[1], args[2], attrs.get("eps", 1e-5))
    if op == "attention":
        # fp32 under h3 math: the h3 flash kernel with per-row scales (a bare
        # attention has no LN-folded weights to bound K / V; the x6 kernel it
        # replaces spends six MFMAs per product instead of three)
        h3 = (args[0].is_cuda and args[0].dtype == torch.float32 and ops.f32_math() == "h3" and not ref
              and os.environ.get("NOS_AMD_BARE_ATTN_X6") != "1")   # (=1: the x6 kernel, for A/B)
        if (attrs.get("causal") or args[0].shape[-1] // (3 * attrs["heads"]) != 64 or not args[0].is_cuda
                or h3):
            from ...ops import tenant as T

            q, k, v = _qkv_views(args[0], attrs["heads"])
            if "q_start" in attrs:
                q = q[:, attrs["q_start"]:attrs["q_end"]]
            return T.sdpa(q, k, v, causal=attrs.get("causal", False), scale=attrs.get("scale")).flatten(2)
        y = ops.attention_qkv(args[0].contiguous(), attrs["heads"], scale=attrs.get("scale"))
        return y[:, attrs["q_start"]:attrs["q_end"]] if "q_start" in attrs else y
    if op == "add":
        return args[0] + args[1]
    if op == "mul":
        return args[0] * args[1]
    if op == "gelu":
        return F.gelu(args[0])
    if op == "relu":
        return F.relu(args[0])
    if op == "sigmoid":
        return torch.sigmoid(args[0])
    if op == "silu":
        return F.silu(args[0])
    if op == "cat":
        return torch.cat(args, dim=attrs["dim"])
    if op == "slice":
        d = attrs["dim"]
        return args[0].narrow(d, attrs["start"], attrs["end"] - attrs["start"])
    if op == "reshape":
        return args[0].reshape(attrs["shape"])
    if op == "permute":
        return args[0].permute(attrs["dims"])
    if op == "expand":
        return args[0].expand(attrs["shape"])
    if op == "cast":
        return args[0].to(torch_dtype(attrs["dtype"]))
    if op == "interpolate":
        mode = attrs.get("mode", "bicubic")
        return F.interpolate(args[0], size=tuple(attrs["size"]), mode=mode,
                             align_corners=None if mode == "nearest" else False)
    if op == "sub":
        return args[0] - args[1]
    if op == "div":
        return args[0] / args[1]
    if op == "tanh":
        return torch.tanh(args[0])
    if op == "exp":
        return torch.exp(args[0])
    if op == "neg":
        return -args[0]
    if op == "rsqrt":
        return torch.rsqrt(args[0])
    if op == "conv2d":
        return F.conv2d(args[0], args[1], args[2] if len(args) > 2 else None, _pair2(attrs, "stride", 1),
                        _pair2(attrs, "padding", 0), _pair2(attrs, "dilation", 1), attrs.get("groups", 1))
    if op == "batchnorm":
        return F.batch_norm(args[0], args[3], args[4], args[1], args[2], False, 0.0, attrs.get("eps", 1e-5))
    if op == "max_pool2d":
        k = _pair2(attrs, "kernel", 1)
        return F.max_pool2d(args[0], k, attrs.get("stride") and _pair2(attrs, "stride", 1) or k,
                            _pair2(attrs, "padding", 0))
    if op == "avg_pool2d":
        k = _pair2(attrs, "kernel", 1)
        return F.avg_pool2d(args[0], k, attrs.get("stride") and _pair2(attrs, "stride", 1) or k,
                            _pair2(attrs, "padding", 0))
    if op == "mean":
        return args[0].mean(dim=attrs["dims"], keepdim=attrs.get("keepdim", False))
    if op == "sum":
        return args[0].sum(dim=attrs["dims"], keepdim=attrs.get("keepdim", False))
    if op == "matmul":
        return args[0] @ args[1]
    if op == "softmax":
        return torch.softmax(args[0].float(), dim=-1).to(args[0].dtype)
    if op == "embedding":
        return F.embedding(args[0].long(), args[1])
    from ...ops import tenant as T

    if op == "rmsnorm":
        return T.rmsnorm_ref(args[0], args[1], attrs.get("eps", 1e-5))
    if op == "rotary":
        return T.rope_ref(args[0], args[1], args[2])
    if op == "sdpa":
        return T.sdpa_ref(args[0], args[1], args[2], attrs.get("causal", False), attrs.get("scale"))
    if op == "kv_write":
        return kv_write_ref(args[0], args[1], args[2])
    if op == "sdpa_cache":
        return sdpa_cache_ref(args[0], args[1], args[2], args[3], attrs.get("scale"))
    if op == "rotary_at":
        return rotary_at_ref(args[0], args[1], args[2], args[3])
    if op == "pos_add":
        return args[0].add_(int(attrs["n"]))
    if op == "pos_set":
        return args[0].fill_(int(attrs["value"]))
    if op == "argmax":
        return args[0].float().argmax(dim=-1).to(torch.int32)
    raise ProgramError(f"op {op!r}")


def kv_write_ref(cache, x, pos):
    """cache[b, pos[b] + i] = x[b, i] for the rows that fit (in place)."""
    L, S = cache.shape[1], x.shape[1]
    for b in range(cache.shape[0]):
        p0 = int(pos[b])
        n = max(0, min(S, L - p0))
        if p0 >= 0 and n:
            cache[b, p0:p0 + n] = x[b, :n].to(cache.dtype)
    return cache


def sdpa_cache_ref(q, kc, vc, pos, scale=None):
    """Query i of sequence b at position pos[b] + i attends the cached keys
    0 .. min(pos[b] + i, L - 1) (fp32 math; grouped-query K / V heads)."""
    import math

    import torch

    B, Sq, H, D = q.shape
    L, Hkv = kc.shape[1], kc.shape[2]
    kf = kc.float().repeat_interleave(H // Hkv, dim=2)
    vf = vc.float().repeat_interleave(H // Hkv, dim=2)
    sc = scale if scale is not None else 1.0 / math.sqrt(D)
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), kf) * sc
    qpos = pos.to(torch.long).view(B, 1) + torch.arange(Sq).view(1, Sq)            # [B, Sq]
    keep = torch.arange(L).view(1, 1, L) <= qpos.clamp(max=L - 1).view(B, Sq, 1)    # [B, Sq, L]
    s = s.masked_fill(~keep[:, None], float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.einsum("bhqk,bkhd->bqhd", p, vf).to(q.dtype)


def rotary_at_ref(x, cos, sin, pos):
    """rotate_half rotary of x [B, S, H, D] at positions pos[b] + i (table
    rows clamped to the table)."""
    import torch

    B, S, H, D = x.shape
    idx = (pos.to(torch.long).view(B, 1) + torch.arange(S).view(1, S)).clamp(0, cos.shape[0] - 1)   # [B, S]
    c = cos.float()[idx][:, :, None, :]
    sn = sin.float()[idx][:, :, None, :]
    xf = x.float()
    rot = torch.cat([-xf[..., D // 2:], xf[..., :D // 2]], dim=-1)
    return (xf * c + rot * sn).to(x.dtype)


def _pair2(attrs: dict, key: str, default: int) -> tuple[int, int]:
    v = attrs.get(key, default)
    return (v, v) if isinstance(v, int) else (v[0], v[1])


def _qkv_views(qkv, heads: int):
    """q, k, v [B, S, H, D] views of a fused projection [B, S, 3*H*D]."""
    B, S, n = qkv.shape
    return qkv.view(B, S, 3, heads, n // (3 * heads)).unbind(2)

