"""Training tenants on the pod server: a program's graph as a trainable module.

The reference's MPS clients are arbitrary CUDA processes, so a fine-tuning
job can share a GPU the same way an inference pod does
(``/root/reference/docs/en/docs/dynamic-gpu-partitioning/partitioning-modes-comparison.md:29-34``).
Inference tenants here are programs lowered onto the gfx950 kernels
(program.py); a *training* tenant registers the same kind of program plus a
training spec, and the server runs whole optimisation steps for it in the
shared context:

* **Model.**  :class:`ProgramModule` evaluates the program's nodes in plain
  PyTorch (``program._eager``: F.linear / F.layer_norm / F.conv2d / softmax
  attention ... -- differentiable, hipBLASLt for the GEMMs) over fp32 master
  weights held as ``nn.Parameter``s; ``cast`` nodes are identities (a bf16
  program trains in fp32).  Weights that are constants by construction
  (BatchNorm running statistics, rotary tables) stay frozen, as do the
  spec's ``frozen`` names.
* **Step.**  forward -> loss (``mse`` against a float target of the
  output's shape, or ``cross_entropy`` of logits [..., C] against int class
  ids [...]) -> backward -> optimizer step (SGD with (Nesterov) momentum /
  Adam / AdamW, torch.optim, capturable) -- on the GPU captured ONCE into a HIP graph, so
  a step is one graph replay on any lane, like an inference.  The capture's
  warm-up steps are undone (weights restored, optimizer state zeroed in
  place), so the first replayed step is the first real step.
* **State.**  :meth:`Trainer.weights_bytes` returns the current weights in
  the program's payload layout; :meth:`Trainer.checkpoint_bytes` appends the
  optimizer state (:func:`state_keys`), and a ``resume`` spec over that
  payload continues the run step for step (the capture restores the loaded
  state in place after its warm-up).

Memory is bounded like an inference tenant's: a static estimate before
anything is allocated (:func:`train_bytes_estimate`), then the measured peak
of build + capture against the slice.
"""
from __future__ import annotations

import math
import os

from .program import Program, ProgramError, _eager, _qkv_views, _req

LOSSES = ("mse", "cross_entropy")
_STEP_SPLIT = 1 << 24   # a checkpointed step count = hi * 2^24 + lo, both exact in float32
OPTIMIZERS = ("sgd", "adam", "adamw")
SPEC_KEYS = {"loss", "optimizer", "lr", "momentum", "nesterov", "weight_decay", "betas", "eps", "output", "frozen",
             "resume"}


def parse_train_spec(spec, prog: Program) -> dict:
    """Validate a register request's ``train`` spec against the program;
    returns it normalised, with the target's shape and dtype."""
    _req(isinstance(spec, dict), "train must be an object")
    extra = set(spec) - SPEC_KEYS
    _req(not extra, f"unknown train keys {sorted(extra)}")
    loss = spec.get("loss", "mse")
    _req(loss in LOSSES, f"train.loss must be one of {LOSSES}")
    opt = spec.get("optimizer", "sgd")
    _req(opt in OPTIMIZERS, f"train.optimizer must be one of {OPTIMIZERS}")

    def num(key, default, lo, hi):
        v = spec.get(key, default)
        _req(isinstance(v, (int, float)) and not isinstance(v, bool) and math.isfinite(v) and lo <= v <= hi,
             f"train.{key} must be a number in [{lo}, {hi}]")
        return float(v)

    for key in ("resume", "nesterov"):   # strict: bool("false") is True
        _req(isinstance(spec.get(key, False), bool), f"train.{key} must be true or false")
    lr = num("lr", 1e-3, 0.0, 10.0)
    _req(not spec.get("nesterov") or (opt == "sgd" and num("momentum", 0.0, 0.0, 0.999) > 0),
         "train.nesterov needs sgd with momentum > 0")
    _req(lr > 0, "train.lr must be > 0")
    out = spec.get("output", 0)
    _req(isinstance(out, int) and 0 <= out < len(prog.outputs), "train.output must index a program output")
    ov = prog.values[prog.outputs[out]]
    _req(ov.dtype in ("fp32", "bf16"), "the trained output must be a float tensor")
    if loss == "mse":
        tshape, tdt = tuple(ov.shape), "fp32"
    else:
        _req(len(ov.shape) >= 2 and ov.shape[-1] >= 2, "cross_entropy needs logits [..., classes >= 2]")
        tshape, tdt = tuple(ov.shape[:-1]), "i32"
    frozen = spec.get("frozen", [])
    _req(isinstance(frozen, list) and all(isinstance(f, str) and f in prog.params for f in frozen),
         "train.frozen must list program weights")
    betas = spec.get("betas", [0.9, 0.999])
    _req(isinstance(betas, list) and len(betas) == 2
         and all(isinstance(b, (int, float)) and 0 <= b < 1 for b in betas), "train.betas must be two numbers in [0, 1)")
    return {"loss": loss, "optimizer": opt, "lr": lr, "momentum": num("momentum", 0.0, 0.0, 0.999),
            "weight_decay": num("weight_decay", 0.0, 0.0, 1.0), "betas": [float(b) for b in betas],
            "eps": num("eps", 1e-8, 1e-12, 1.0), "output": out, "frozen": sorted(set(frozen) | constant_weights(prog)),
            "resume": bool(spec.get("resume", False)), "nesterov": bool(spec.get("nesterov", False)),
            "target_shape": tshape, "target_dtype": tdt}


def constant_weights(prog: Program) -> set[str]:
    """Weights that are constants of the architecture, not learnable:
    BatchNorm running mean / variance and rotary tables."""
    out = set()
    for n in prog.nodes:
        if n.op == "batchnorm":
            out.update(i for i in n.inputs[3:5] if i in prog.params)
        elif n.op == "rotary":
            out.update(i for i in n.inputs[1:3] if i in prog.params)
    return out


def train_bytes_estimate(prog: Program, spec: dict) -> int:
    """Device bytes a training tenant needs, bounded before allocation:
    fp32 master weights + gradients + optimizer state (1 buffer for SGD with
    momentum, 2 for AdamW), the input and target, and every node's output
    kept for the backward pass twice over (activations and their gradients,
    plus the capture's private pool)."""
    w = sum(v.numel * 4 for v in prog.params.values())
    trainable = sum(v.numel * 4 for k, v in prog.params.items() if k not in spec["frozen"])
    states = {"sgd": 1 if spec["momentum"] > 0 else 0, "adam": 2, "adamw": 2}[spec["optimizer"]]
    acts = sum(prog.values[n.output].numel * 4 for n in prog.nodes)
    # the differentiable attention materialises its B x H x Sq x Skv scores: the
    # scores, the masked copy and the probabilities are kept for backward --
    # a long-sequence spec is refused here, not at capture
    # (train_ops.ChunkedAttention: per layer the saved log-sum-exp rows, the live
    # scores of one query chunk at a time; NOS_AMD_TRAIN_NATIVE=0: the full
    # B x H x Sq x Skv scores, masked copy and probabilities of every layer)

    from .train_ops import scores_bytes

    native = os.environ.get("NOS_AMD_TRAIN_NATIVE", "1") != "0"
    scores = live = 0
    for n in prog.nodes:
        if n.op == "sdpa":
            (b, sq, h, _), skv = prog.values[n.inputs[0]].shape, prog.values[n.inputs[1]].shape[1]
        elif n.op == "attention":
            b, sq, _ = prog.values[n.inputs[0]].shape
            h, skv = n.attrs["heads"], sq
        else:
            continue
        if native:
            scores += 4 * b * h * sq
            live = max(live, scores_bytes(b, h, sq, skv))
        else:
            scores += 3 * b * h * sq * skv * 4
    scores += live
    tgt = math.prod(spec["target_shape"]) * 4
    return (w + trainable * (1 + states) + sum(v.numel * 4 for v in prog.inputs) + tgt + 2 * acts
            + 2 * scores)


def _train_op(op: str, args: list, attrs: dict):
    """One node, differentiable: GEMMs and attention on the gfx950 kernels
    (train_ops: h3 GEMMs for the forward and both backward products, chunked
    attention with a log-sum-exp recompute -- no S x S scores kept), the rest
    in PyTorch.  ``NOS_AMD_TRAIN_NATIVE=0``: PyTorch throughout (A/B)."""

    native = os.environ.get("NOS_AMD_TRAIN_NATIVE", "1") != "0"
    if op == "attention":
        from ..ops import tenant as T
        from . import train_ops

        q, k, v = _qkv_views(args[0], attrs["heads"])
        if "q_start" in attrs:
            q = q[:, attrs["q_start"]:attrs["q_end"]]
        if native:
            return train_ops.attention(q, k, v, attrs.get("causal", False), attrs.get("scale")).flatten(2)
        return T.sdpa_ref(q, k, v, attrs.get("causal", False), attrs.get("scale")).flatten(2)
    if op == "sdpa" and native:
        from . import train_ops

        return train_ops.attention(args[0], args[1], args[2], attrs.get("causal", False), attrs.get("scale"))
    if op == "linear" and native:
        import torch.nn.functional as F

        from . import train_ops

        y = train_ops.linear(args[0], args[1], args[2] if len(args) > 2 else None)
        act = attrs.get("act")
        return F.gelu(y) if act == "gelu" else (F.relu(y) if act == "relu" else y)
    if op == "cast":
        return args[0]  # fp32 master copy: a bf16 program trains in fp32
    return _eager(op, args, attrs, ref=True)


def _module_cls():
    import torch.nn as nn

    class ProgramModule(nn.Module):
        """A program's graph as a module over its weights (fp32 Parameters,
        frozen ones as buffers)."""

        def __init__(self, prog: Program, params: dict, frozen):
            super().__init__()
            self.prog = prog
            self.slots: dict[str, tuple[str, int]] = {}
            self.weights = nn.ParameterList()
            fixed = []
            for name in prog.params:
                t = params[name].detach().float().clone()
                if name in frozen:
                    self.slots[name] = ("b", len(fixed))
                    fixed.append(t)
                else:
                    self.slots[name] = ("p", len(self.weights))
                    self.weights.append(nn.Parameter(t))
            for i, t in enumerate(fixed):
                self.register_buffer(f"fixed{i}", t)

        def weight(self, name: str):
            kind, i = self.slots[name]
            return self.weights[i] if kind == "p" else getattr(self, f"fixed{i}")

        def forward(self, x):
            env = {name: self.weight(name) for name in self.prog.params}
            env[self.prog.inputs[0].name] = x if self.prog.inputs[0].dtype == "i32" else x.float()
            for n in self.prog.nodes:
                env[n.output] = _train_op(n.op, [env[i] for i in n.inputs], n.attrs)
            return tuple(env[o] for o in self.prog.outputs)

    return ProgramModule


def state_keys(spec: dict) -> list[str]:
    """The optimizer state a checkpoint carries per trainable weight, in
    order: SGD's momentum buffer (with momentum), AdamW's two moments + step."""
    if spec["optimizer"] == "sgd":
        return ["momentum_buffer"] if spec["momentum"] > 0 else []
    return ["exp_avg", "exp_avg_sq", "step"]


def state_nbytes(prog: Program, spec: dict) -> int:
    """Bytes of the optimizer-state block that follows the weights in a
    resume payload (fp32, weight by weight in program order)."""
    keys = state_keys(spec)
    per = sum(v.numel for k, v in prog.params.items() if k not in spec["frozen"])
    n = sum(1 for k in prog.params if k not in spec["frozen"])
    # Adam's step: two float32 slots, hi * 2^24 + lo, exact past 2^24 steps
    return 4 * (per * sum(1 for k in keys if k != "step") + 2 * n * ("step" in keys))


class Trainer:
    """Optimisation steps of one training tenant (see the module docstring)."""

    def __init__(self, prog: Program, spec: dict, device, state: bytes | None = None):
        import torch

        self.prog, self.spec = prog, spec
        self.device = torch.device(device)
        self.module = _module_cls()(prog, prog.tensors(self.device), set(spec["frozen"])).to(self.device)
        ps = list(self.module.weights)
        cap = self.device.type == "cuda"
        if spec["optimizer"] == "sgd":
            self.opt = torch.optim.SGD(ps, lr=spec["lr"], momentum=spec["momentum"], nesterov=spec["nesterov"],
                                       weight_decay=spec["weight_decay"], foreach=True)
        else:
            cls = torch.optim.AdamW if spec["optimizer"] == "adamw" else torch.optim.Adam
            self.opt = cls(ps, lr=spec["lr"], betas=tuple(spec["betas"]), eps=spec["eps"],
                           weight_decay=spec["weight_decay"], capturable=cap, foreach=True)
        self.x = prog.input_tensor(self.device)
        tdt = torch.int64 if spec["target_dtype"] == "i32" else torch.float32
        self.y = torch.zeros(spec["target_shape"], dtype=tdt, device=self.device)
        self.graph = None
        self.loss = None
        self.steps = 0
        self._resume = None
        if state is not None:
            self._load_state(state)

    def _load_state(self, raw: bytes) -> None:
        """Optimizer state from a checkpoint (:meth:`checkpoint_bytes`), set
        before the first step -- the optimizers then continue from it."""
        import numpy as np
        import torch

        if len(raw) != state_nbytes(self.prog, self.spec):
            raise ProgramError(f"optimizer state of {len(raw)} bytes, the spec needs "
                               f"{state_nbytes(self.prog, self.spec)}")
        a = np.frombuffer(raw, dtype=np.float32)
        off = 0
        cap = self.device.type == "cuda"
        saved = {}
        for p in self.module.weights:
            st = {}
            for k in state_keys(self.spec):
                if k == "step":
                    v = torch.tensor(float(int(a[off]) * _STEP_SPLIT + int(a[off + 1])), dtype=torch.float32)
                    st[k] = v.to(self.device) if cap else v
                    off += 2
                else:
                    st[k] = torch.from_numpy(a[off:off + p.numel()].copy()).view(p.shape).to(self.device)
                    off += p.numel()
            if st:
                self.opt.state[p] = st
                saved[p] = {k: v.clone() for k, v in st.items()}
        self._resume = saved

    def checkpoint_bytes(self) -> bytes:
        """Weights (payload layout) followed by the optimizer state: a
        register payload for ``train={..., "resume": True}``."""
        import numpy as np

        parts = [self.weights_bytes()]
        for p in self.module.weights:
            st = self.opt.state.get(p, {})
            for k in state_keys(self.spec):
                v = st.get(k)
                if k == "step":
                    n = int(round(float(v))) if v is not None else 0
                    parts.append(np.asarray(divmod(n, _STEP_SPLIT), np.float32).tobytes())
                else:
                    t = v.detach().float().cpu().numpy() if v is not None else np.zeros(p.shape, np.float32)
                    parts.append(np.ascontiguousarray(t, dtype=np.float32).tobytes())
        return b"".join(parts)

    def _loss(self):
        import torch.nn.functional as F

        out = self.module(self.x)[self.spec["output"]].float()
        if self.spec["loss"] == "mse":
            return F.mse_loss(out, self.y)
        if out.is_cuda and os.environ.get("NOS_AMD_TRAIN_NATIVE", "1") != "0":
            from .train_ops import cross_entropy

            return cross_entropy(out.reshape(-1, out.shape[-1]), self.y.reshape(-1))
        return F.cross_entropy(out.reshape(-1, out.shape[-1]), self.y.reshape(-1))

    def _eager_step(self):
        self.opt.zero_grad(set_to_none=True)
        loss = self._loss()
        loss.backward()
        self.opt.step()
        return loss.detach()

    def capture(self, stream, warmup: int = 2) -> None:
        """Capture forward + backward + optimizer step into one graph on
        ``stream``; the warm-up steps' effects are undone in place."""
        import torch

        saved = [p.detach().clone() for p in self.module.weights]
        with torch.cuda.stream(stream):
            for _ in range(warmup):
                self._eager_step()
            stream.synchronize()
            with torch.no_grad():
                for p, s in zip(self.module.weights, saved):
                    p.copy_(s)
                for p, st in self.opt.state.items():   # in place: the graph keeps the addresses
                    for k, v in st.items():
                        if torch.is_tensor(v):
                            if self._resume is not None and p in self._resume:
                                v.copy_(self._resume[p][k])   # the checkpoint's state
                            else:
                                v.zero_()                      # a fresh optimizer
            self.opt.zero_grad(set_to_none=True)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream, capture_error_mode="thread_local"):
                self.loss = self._loss()
                self.loss.backward()
                self.opt.step()
            stream.synchronize()
        self.graph = g

    def step(self, x=None, y=None):
        """One optimisation step on (x, y) (None: keep the resident tensors);
        returns the loss tensor (before the step's update).  Stream-ordered
        on the GPU: the caller synchronises."""
        import torch

        if x is not None:
            self.x.copy_(torch.as_tensor(x).view(self.x.shape).to(self.x.dtype))
        if y is not None:
            self.y.copy_(torch.as_tensor(y).view(self.y.shape).to(self.y.dtype))
        self.steps += 1
        if self.graph is not None:
            self.graph.replay()
            return self.loss
        return self._eager_step()

    def forward(self, x=None) -> tuple:
        import torch

        with torch.no_grad():
            if x is not None:
                self.x.copy_(torch.as_tensor(x).view(self.x.shape).to(self.x.dtype))
            return self.module(self.x)

    def weights_bytes(self) -> bytes:
        """The current weights in the program's payload layout (each in its
        wire dtype): a register payload that resumes from here."""
        import numpy as np
        import torch

        buf = bytearray(max((off + nb for off, nb in self.prog.param_layout.values()), default=0))
        for name, v in self.prog.params.items():
            off, nb = self.prog.param_layout[name]
            t = self.module.weight(name).detach()
            if v.dtype == "bf16":
                raw = t.to(torch.bfloat16).view(torch.int16).cpu().numpy().tobytes()
            else:
                raw = t.float().cpu().numpy().astype(np.float32).tobytes()
            if len(raw) != nb:
                raise ProgramError(f"weight {name!r}: {len(raw)} bytes for a {nb}-byte span")
            buf[off:off + nb] = raw
        return bytes(buf)
