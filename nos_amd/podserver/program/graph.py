"""A validated program (:class:`Program`): its device-memory accounting
(the static estimate the server checks against the slice before a build),
its weights as tensors, and the entry points to the compiler and the eager
reference."""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .ir import GEMM_OPS, NEVER_FOLD, Node, Value, torch_dtype
from .reference import _eager

def _workspace(node: Node, ins: list[Value], out: Value, f32_math: str) -> int:
    """Transient device bytes one op allocates while it runs, beyond its
    inputs and output (an upper bound; :meth:`Program.bytes_estimate_for`)."""
    op = node.op
    if op == "linear" and ins[0].dtype == "fp32" and f32_math == "h3":
        m = ins[0].numel // ins[0].shape[-1]
        return ins[0].nbytes + 4 * m                       # A's fp16 planes + row scales
    if op == "linear_rms" or (op == "linear" and ins[0].dtype == "bf16" and f32_math == "h3"):
        m = ins[0].numel // ins[0].shape[-1]
        return 2 * m * ins[0].shape[-1] * 4 + 4 * m + out.numel * 4
    if op == "attention":
        b, s, three_hd = ins[0].shape
        h = node.attrs["heads"]
        return _attn_ws(b, s, s, h, h, three_hd // (3 * h)) + ins[0].nbytes + out.numel * 4
    if op == "sdpa":
        (b, sq, h, d), (_, skv, hkv, _) = ins[0].shape, ins[1].shape
        copies = sum(v.numel * 4 for v in ins[:3]) if ins[0].dtype != "fp32" else 0
        return _attn_ws(b, sq, skv, h, hkv, d) + copies + out.numel * 4
    if op == "conv2d":
        n, c, _, _ = ins[0].shape
        oc, cg, kh, kw = ins[1].shape
        p = out.numel // (n * oc)
        kp = -(-(cg * kh * kw) // 32) * 32
        return n * (c // cg) * p * (kp * 4 + 4) + ins[0].numel * 4 + out.numel * 4
    if op == "matmul":
        k = ins[0].shape[-1]
        kp = -(-k // 32) * 32
        rows = ins[0].numel // k + ins[1].numel // k
        return rows * kp * 12 + out.numel * 4          # padded fp32 copies + planes + the fp32 result
    return 0


def _attn_ws(b: int, sq: int, skv: int, h: int, hkv: int, d: int) -> int:
    """Upper bound of both attention kernels' workspaces (attention_f32x.hip
    nos_attn_f32x6_workspace, attention_h3g.hip nos_attn_h3g_workspace)."""
    skvp = -(-skv // 32) * 32
    return b * max(h, hkv) * skvp * 6 * d * 2 + 4 * b * sq * h * (d + 2) * 4 + b * hkv * (skv // 256 + 2) * 8 + 4096



@dataclass
class Program:
    name: str
    inputs: list[Value]
    params: dict[str, Value]
    param_layout: dict[str, tuple[int, int]]     # name -> (offset, nbytes) in the payload
    nodes: list[Node]
    outputs: list[str]
    values: dict[str, Value]
    payload: bytes | memoryview = b""
    state: dict[str, Value] = field(default_factory=dict)        # persistent buffers (K / V caches, positions)
    state_root: dict[str, str] = field(default_factory=dict)     # a state's in-place versions -> the state

    # ------------------------------------------------------------ accounting
    @property
    def param_bytes(self) -> int:
        return sum(v.nbytes for v in self.params.values())

    @property
    def state_bytes(self) -> int:
        return sum(v.nbytes for v in self.state.values())

    def is_state(self, name: str) -> bool:
        """A state buffer or one of its in-place versions (the same memory)."""
        return name in self.state or name in self.state_root

    @property
    def bytes_estimate(self) -> int:
        return self.bytes_estimate_for(None)

    def foldable(self) -> set[str]:
        """Node outputs the compiler folds to constants at load time (every
        input a weight or another folded value; never attention)."""
        const = set(self.params)
        out = set()
        for n in self.nodes:
            if n.op not in NEVER_FOLD and all(i in const for i in n.inputs):
                const.add(n.output)
                out.add(n.output)
        return out

    def bytes_estimate_for(self, kernel_config: dict | None = None) -> int:
        """Device bytes a build needs, bounded before anything is allocated:

        * the weights, plus their split planes under the server's fp32 math
          (``kernel_config["f32_math"]``; h3: two fp16 planes = 1x an fp32
          matrix + row scales; x6: three bf16 planes = 1.5x; exact: none) and
          the folded copy LayerNorm / RMSNorm folding makes of a weight
          (+ its two bias vectors);
        * constant-folded values, which are weights too: they are counted as
          persistent (they are materialised at load time and live
          for the tenant's lifetime), never released;
        * the input, and the peak of the unfused graph's live activations
          when every value is released after its last consumer (what the
          compiled program does; fusion only removes intermediates) plus the
          largest per-op workspace live at that point (GEMM A planes, the
          attention's K/V planes, conv im2col planes, ...; :func:`_workspace`),
          twice over: one graph plus the solo graph's private buffers.

        The measured peak of the real build is checked again after it."""
        f32_math = (kernel_config or {}).get("f32_math", "h3")
        folded = self.foldable()
        persistent = sum(self.values[o].nbytes for o in folded)
        last = {}
        for k, n in enumerate(self.nodes):
            for i in n.inputs:
                last[i] = k
        keep = set(self.outputs)
        live = peak = 0
        for k, n in enumerate(self.nodes):
            if n.output in folded:
                continue
            ws = _workspace(n, [self.values[i] for i in n.inputs], self.values[n.output], f32_math)
            if not self.is_state(n.output):   # an in-place state update allocates nothing
                live += self.values[n.output].nbytes
            peak = max(peak, live + ws)
            for i in set(n.inputs):
                v = self.values[i]
                if (v.kind == "node" and i not in folded and last.get(i) == k and i not in keep
                        and not self.is_state(i)):
                    live -= v.nbytes
        plane_mult = {"h3": 1.0, "x6": 1.5}.get(f32_math, 0.0)
        planes = 0
        by_out = {n.output: n for n in self.nodes}
        for n in self.nodes:
            if n.op not in GEMM_OPS or len(n.inputs) < 2 or n.inputs[1] not in self.params:
                continue
            w = self.values[n.inputs[1]]
            if w.dtype == "fp32":
                planes += int(w.nbytes * plane_mult) + 4 * w.shape[0]
            src = by_out.get(n.inputs[0])
            if src is not None and src.op in ("layernorm", "rmsnorm"):  # the folded copy + c1 / c2
                planes += w.nbytes + 8 * w.shape[0]
        # parallel linears over one activation (Q / K / V, gate / up, heads) are merged into one
        # weight copy by the compiler (not only the norm-fed ones)
        readers: dict[str, list] = {}
        for n in self.nodes:
            if n.op == "linear" and len(n.inputs) >= 2 and n.inputs[1] in self.params:
                readers.setdefault(n.inputs[0], []).append(self.values[n.inputs[1]])
        for ws in readers.values():
            if len(ws) > 1:
                planes += sum(w.nbytes + 4 * w.shape[0] for w in ws)
        # the state (K / V caches, positions) is allocated once, at registration,
        # and never grows at replay: it counts in full against the slice
        return (self.param_bytes + planes + persistent + self.state_bytes + sum(v.nbytes for v in self.inputs)
                + 2 * peak)

    # ------------------------------------------------------------ tensors
    def tensors(self, device) -> dict:
        """The weights as device tensors (copied out of the payload)."""
        import torch

        out = {}
        buf = memoryview(self.payload)
        for name, v in self.params.items():
            off, nb = self.param_layout[name]
            raw = np.frombuffer(buf[off:off + nb], dtype=np.float32 if v.dtype == "fp32" else np.int16)
            t = torch.from_numpy(raw.copy()).view(v.shape)
            if v.dtype == "bf16":
                t = t.view(torch.bfloat16)
            out[name] = t.to(device)
        return out

    def state_tensors(self, device) -> dict:
        """The state buffers, zero-initialised (a fresh sequence at position 0)."""
        import torch

        return {k: torch.zeros(v.shape, dtype=torch_dtype(v.dtype), device=device) for k, v in self.state.items()}

    def input_tensor(self, device, data: np.ndarray | None = None):
        import torch

        v = self.inputs[0]
        if data is None:
            x = torch.zeros(v.shape, dtype=torch_dtype(v.dtype))
        elif v.dtype == "i32":
            x = torch.from_numpy(np.ascontiguousarray(data, dtype=np.int32)).view(v.shape)
        else:
            x = torch.from_numpy(np.ascontiguousarray(data, dtype=np.float32)).view(v.shape).to(torch_dtype(v.dtype))
        return x.to(device)

    def id_bound(self) -> int | None:
        """For an i32 (token id) input: the smallest embedding table it
        indexes -- ids must lie in [0, bound) (checked per request)."""
        if self.inputs[0].dtype != "i32":
            return None
        vs = [self.values[n.inputs[1]].shape[0] for n in self.nodes if n.op == "embedding"]
        return min(vs) if vs else None

    # ------------------------------------------------------------ execution
    def compile(self, device, params: dict | None = None, state: dict | None = None,
                derived: dict | None = None) -> "CompiledProgram":  # noqa: F821
        """``state``: the tenant's state tensors (:meth:`state_tensors`), shared
        by every variant compiled over them; None: fresh zero buffers.
        ``derived``: a dict shared by the variants compiled over the same
        ``params`` -- their folded / merged weights are then made once."""
        from .execute import CompiledProgram

        return CompiledProgram(self, device, params, state, derived)

    def reference(self, x, params: dict | None = None, state: dict | None = None) -> tuple:
        """Eager, unfused, fp32 evaluation of the graph on the CPU (the
        numerics reference: every op in plain PyTorch).  ``state``: the
        tenant's state tensors (fp32 / i32 on the CPU), updated in place --
        pass the same dict to consecutive calls (prefill, then decode steps);
        None: a fresh zero state, dropped after the call."""
        import torch

        ps = params if params is not None else self.tensors("cpu")
        env = {k: t.float().cpu() for k, t in ps.items()}
        if state is None:
            state = {k: (t if t.dtype == torch.int32 else t.float()) for k, t in self.state_tensors("cpu").items()}
        env.update(state)
        env[self.inputs[0].name] = x.cpu() if self.inputs[0].dtype == "i32" else x.float().cpu()
        with torch.no_grad():
            for n in self.nodes:
                args = [env[i] for i in n.inputs]
                if n.op == "cast":
                    env[n.output] = args[0]
                else:
                    env[n.output] = _eager(n.op, args, n.attrs, ref=True)
        return tuple(env[o] for o in self.outputs)

