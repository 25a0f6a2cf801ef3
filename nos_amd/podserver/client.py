"""Fractional pod side of the pod server (server.py): stdlib + numpy only.

A pod scheduled onto a pod-server slice gets, from the device plugin,
``NOS_AMD_POD_SERVER`` (its GPU's server socket, in the one per-GPU directory
the container mounts), ``NOS_AMD_POD_TOKEN`` (the allocation's token: the
server reads the slice's memory and CU mask from the plugin's record of it),
``NOS_AMD_MEMORY_LIMIT_GB`` (informational) and no ``/dev/kfd`` or render
node.  The container never opens the GPU.  It registers its model once -- a
program (op graph + weights, program.py) -- then sends inference requests.
This is the role MPS clients play in the reference: their CUDA calls go to
the MPS server, which runs them in the server's context.

Server loss.  A request whose connection breaks raises
:class:`PodServerGone` (the pod exits non-zero and the kubelet restarts it),
unless the client was made with ``reconnect_s`` > 0: it then waits up to that
long for the server (the supervisor restarts a dead one), registers the same
program again with the same token, and retries the request once.
"""
from __future__ import annotations

import os
import socket
import time

import numpy as np

from ..api.constants import ENV_MEMORY_LIMIT_GB, ENV_POD_CU_MASK, ENV_POD_SERVER, ENV_POD_TOKEN
from . import protocol as P


class PodServerError(RuntimeError):
    pass


class PodServerGone(PodServerError):
    """The connection to the pod server broke (server died or evicted us)."""


def _connect(path: str, timeout_s: float) -> socket.socket:
    deadline = time.monotonic() + timeout_s
    while True:  # the server's socket appears once it accepts (server.start)
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        try:
            s.connect(path)
            return s
        except (FileNotFoundError, ConnectionRefusedError):
            s.close()
            if time.monotonic() > deadline:
                raise PodServerError(f"no pod server at {path} after {timeout_s} s")
            time.sleep(0.1)


def _wire(a, want: str | None, what: str) -> np.ndarray:
    """``a`` as the bytes the tenant reads: the registered program's type
    (``want``, from the register reply) decides, not the array's -- a uint8
    image or an int arange for an fp32 model goes as float32 values.  Float
    data for an id input is refused rather than truncated.  Without ``want``
    (no register reply seen) integer arrays go as int32, others as float32."""
    a = np.asarray(a)
    is_int = np.issubdtype(a.dtype, np.integer) or a.dtype == np.bool_
    if want == "i32":
        if not is_int:
            raise PodServerError(f"{what}: the tenant's model takes integer ids, got {a.dtype}")
        return np.ascontiguousarray(a, dtype=np.int32)
    if want == "f32" or not is_int:
        return np.ascontiguousarray(a, dtype=np.float32)
    return np.ascontiguousarray(a, dtype=np.int32)


class PodClient:
    def __init__(self, path: str | os.PathLike, connect_timeout_s: float = 60.0, reconnect_s: float = 0.0):
        self.path = str(path)
        self.sock = _connect(self.path, connect_timeout_s)
        self.reconnect_s = reconnect_s
        self.tenant: int | None = None
        self.info: dict = {}
        self._reg: tuple[dict, bytes] | None = None
        self.input_dtype: str | None = None    # "f32" / "i32": the registered program's input (register reply)
        self.target_dtype: str | None = None   # a training tenant's target
        self.reconnects = 0

    @classmethod
    def from_env(cls, env: dict | None = None, **kw) -> "PodClient":
        env = os.environ if env is None else env
        path = env.get(ENV_POD_SERVER)
        if not path:
            raise PodServerError(f"{ENV_POD_SERVER} is not set: this pod was not allocated a pod-server slice")
        return cls(path, **kw)

    def _call(self, req: dict, payload: bytes = b"", reply_limit: int | None = None) -> tuple[dict, bytes]:
        if self.sock is None:
            raise PodServerGone("client is closed")
        try:
            P.send_msg(self.sock, req, payload)
            rep, data = P.recv_msg(self.sock, None if reply_limit is None else (lambda obj, n: reply_limit))
        except (ConnectionError, OSError) as e:
            raise PodServerGone(f"pod server connection lost: {e}") from e
        if not rep.get("ok"):
            raise PodServerError(rep.get("error", "pod server error"))
        return rep, data

    def register(self, pod: str, program: dict, weights: bytes = b"", token: str | None = None,
                 memory_limit_gb: float | None = None, cu_mask: str | None = None, env: dict | None = None,
                 variants: list[dict] | None = None, train: dict | None = None,
                 priority: str | None = None) -> dict:
        """Ship the pod's program (op graph + weight bytes, program.py) to the
        server.  The allocation token comes from the device plugin's env; the
        slice itself is the plugin's record.  ``memory_limit_gb`` /
        ``cu_mask`` matter only to a server without allocation records.
        ``variants``: the same model's programs for other input shapes (over
        the same ``weights``); :meth:`infer` routes by the input's shape.
        ``train``: register a training tenant (podserver/training.py: loss,
        optimizer, lr, ...) driven by :meth:`train_step`."""
        env = os.environ if env is None else env
        if memory_limit_gb is None and env.get(ENV_MEMORY_LIMIT_GB):
            memory_limit_gb = float(env[ENV_MEMORY_LIMIT_GB])
        req = {"op": "register", "pod": pod, "program": program, "token": token or env.get(ENV_POD_TOKEN),
               "memory_limit_gb": memory_limit_gb, "cu_mask": cu_mask or env.get(ENV_POD_CU_MASK)}
        if variants:
            req["variants"] = list(variants)
        if train is not None:
            req["train"] = dict(train)
        if priority is not None:   # "latency": the server's priority lanes (default for stateful programs)
            req["priority"] = priority
        rep, _ = self._call(req, weights)
        self._reg = (req, weights)
        self.input_dtype = rep.get("input_dtype")
        self.target_dtype = rep.get("target_dtype")
        self.tenant = rep["tenant"]
        self.info = rep
        return rep

    def _reregister(self) -> None:
        deadline = time.monotonic() + self.reconnect_s
        last = None
        while time.monotonic() < deadline:
            try:
                self.sock.close()
            except OSError:
                pass
            try:
                self.sock = _connect(self.path, max(0.1, deadline - time.monotonic()))
                rep, _ = self._call(*self._reg)
                self.tenant, self.info = rep["tenant"], rep
                self.reconnects += 1
                return
            except PodServerError as e:  # not up yet / still holding our old tenant: retry
                last = e
                time.sleep(0.2)
        raise PodServerGone(f"pod server did not come back within {self.reconnect_s} s: {last}")

    def infer(self, x: np.ndarray | None = None, outputs: bool | list = False) -> tuple[list[np.ndarray], dict]:
        """One inference on the pod's model; ``x`` replaces the resident input
        (one of the registered input shapes; without ``x`` the primary
        shape's resident input runs).  ``outputs``: return every output
        (True), none, or those of the listed indices.  A stateful tenant's
        reply carries its counters (``rep["state"]``, e.g. the position)."""
        req = {"op": "infer", "outputs": outputs}
        if x is None:
            payload = b""
        else:
            wire = _wire(x, self.input_dtype, "input")
            payload = wire.tobytes()
            req["shape"] = [int(d) for d in np.shape(x)]
            req["dtype"] = "i32" if wire.dtype == np.int32 else "f32"
        try:
            rep, data = self._call(req, payload)
        except PodServerGone:
            if self.reconnect_s <= 0 or self._reg is None:
                raise
            self._reregister()
            rep, data = self._call(req, payload)
        return (P.unpack_arrays(rep["outputs"], data) if outputs else []), rep

    def reset(self) -> dict:
        """Zero a stateful tenant's state (K / V caches, positions): a new
        sequence.  Returns the reply (``state``: the counters, now 0)."""
        return self._call({"op": "reset"})[0]

    def generate(self, prompt: np.ndarray, max_new_tokens: int, next_output: int = -1,
                 server_loop: bool = True) -> tuple[np.ndarray, dict]:
        """Greedy generation on a stateful decoder tenant
        (models/llama_program.llama_decode_programs): the prompt ids [B, P]
        go to the prefill variant, then the decode variant runs once per new
        token, fed the program's next-ids output (``next_output``).
        ``server_loop``: the decode steps run as ONE ``generate`` request --
        the server replays the decode graph back to back, feeding the ids on
        the device, and returns every token at the end (no host round trip
        per token); otherwise one [B, 1] request per token.  Returns (ids [B,
        max_new_tokens], timings: the prefill's round trip, every decode
        step's (server loop: the loop's time / steps), the server's final
        counters)."""
        prompt = np.asarray(prompt)
        B = prompt.shape[0]
        t0 = time.monotonic()
        outs, rep = self.infer(prompt, outputs=[next_output])
        t1 = time.monotonic()
        tok = outs[0].reshape(B, -1)[:, -1].astype(np.int32)
        toks, steps = [tok], []
        n = max_new_tokens - 1
        if server_loop and n > 0:
            wire = _wire(tok.reshape(B, 1), self.input_dtype, "input")
            req = {"op": "generate", "steps": n, "output": next_output, "shape": [B, 1],
                   "dtype": "i32" if wire.dtype == np.int32 else "f32"}
            s0 = time.monotonic()
            rep, data = self._call(req, wire.tobytes())
            dt = time.monotonic() - s0
            ids = P.unpack_arrays(rep["outputs"], data)[0].reshape(n, B, -1)[:, :, -1].astype(np.int32)
            toks += list(ids)
            steps = [dt / n] * n
        else:
            for _ in range(n):
                s0 = time.monotonic()
                outs, rep = self.infer(tok.reshape(B, 1), outputs=[next_output])
                steps.append(time.monotonic() - s0)
                tok = outs[0].reshape(B, -1)[:, -1].astype(np.int32)
                toks.append(tok)
        return np.stack(toks, axis=1), {"prefill_s": t1 - t0, "step_s": steps, "state": rep.get("state")}

    def train_step(self, x: np.ndarray, target: np.ndarray) -> dict:
        """One optimisation step of a training tenant on (x, target): the
        target has the trained output's shape (mse, float) or its shape
        without the class dim (cross_entropy, int class ids).  Returns the
        reply: ``loss`` (before the step's update), ``step``, timings."""
        xa = _wire(x, self.input_dtype, "input")
        ta = _wire(target, self.target_dtype, "target")
        xb = xa.tobytes()
        return self._call({"op": "train", "x_bytes": len(xb), "dtype": "i32" if xa.dtype == np.int32 else "f32",
                           "target_dtype": "i32" if ta.dtype == np.int32 else "f32"}, xb + ta.tobytes())[0]

    def weights(self) -> bytes:
        """A training tenant's current weights in its program's payload
        layout: ``register(program, weights=...)`` resumes from them."""
        # a weight payload may exceed the protocol's default 1 GiB reply bound
        # (the server's slice bounds it); the caller asked for all of it
        return self._call({"op": "weights"}, reply_limit=1 << 42)[1]

    def checkpoint(self) -> bytes:
        """A training tenant's weights followed by its optimizer state:
        ``register(program, weights=<this>, train={..., "resume": True})``
        continues the run where it stopped."""
        return self._call({"op": "checkpoint"}, reply_limit=1 << 42)[1]

    def stats(self) -> dict:
        return self._call({"op": "stats"})[0]

    def close(self) -> None:
        if self.sock is None:
            return
        try:
            self._call({"op": "close"})
        except (OSError, PodServerError, ConnectionError):
            pass
        self.sock.close()
        self.sock = None


__all__ = ["PodClient", "PodServerError", "PodServerGone", "ENV_POD_SERVER", "ENV_POD_CU_MASK", "ENV_POD_TOKEN"]
