"""nos-amd pod server: the MI355X stand-in for the NVIDIA MPS control daemon.

Why it exists.  The reference shares a GPU between up to 48 client pods through
MPS (``pkg/gpu/slicing``; the nvidia-device-plugin starts the MPS daemon): the
clients' kernels run in ONE server context.  AMD has no MPS.  Separate pod
processes on one MI355X each take a KFD process slot of the amdgpu hardware
scheduler, which runs at most 8 of them at once (``gpu/kfd.py``); a ninth is
time-sliced at a ~50 ms quantum and aggregate throughput falls
(profiles/r02_pods_vs_throughput_hwqueues.json).  The pod server removes that
bound the way MPS does on NVIDIA.  One server process per GPU owns the only
HIP context.  Fractional pods are CPU-only clients (``client.py``) on a Unix
socket, and their inferences run as HIP-graph replays in the server.

Design (MI355X-first):

* **Lanes.**  ``lanes`` HIP streams are created first, so that with
  ``GPU_MAX_HW_QUEUES=lanes`` each one owns a hardware queue.  Every tenant's
  graph is replayed on whichever lane is free.  A CUDA/HIP graph may be
  launched on any stream, so tenants do not need their own queue; 28 tenants
  on 28 queues oversubscribe the command processor's queue slots and lose
  throughput (tools/mps_probe.py: 323-421 inf/s at 28 tenants with 8-32
  queues, against 476 at 8 and 16 tenants on their own queues).
* **Fairness.**  Requests enter one FIFO and each client has at most one
  request in flight, so the lanes serve the tenants round-robin and every
  tenant sees the same latency.  Queues shared through HIP's round-robin
  stream mapping instead gave a 20-50 ms spread at 20 tenants.
* **Programs.**  A tenant ships its model as a program -- a static op graph
  over the whitelisted nos-amd ops plus raw weight bytes (program.py) -- not
  code.  The server validates it (shapes, dtypes, kernel constraints), lowers
  it with its small graph compiler (constant folding, LayerNorm folding,
  epilogue and QKV-attention fusion) onto the gfx950 kernels, and captures it
  into HIP graphs like any model.
* **Admission.**  With an allocations directory (the deployed default), a
  tenant registers with the per-allocation token the device plugin minted
  (``NOS_AMD_POD_TOKEN``); its slice memory and CU mask come from the
  plugin's record, never from the client, one tenant per token, and a
  tenant whose record disappears (its pod's devices were released) is
  evicted (allocations.py).  Memory is checked twice, both hard: the
  program's static estimate before anything is allocated, then the measured
  peak device memory of the build and graph capture.  Slots and memory are
  reserved under the lock before the (slow) build, so concurrent
  registrations cannot over-commit.  Nothing is allocated at replay time.
  Process pods only get a cooperative caching-allocator cap.
* **CU slices.**  A tenant whose allocation carries a CU mask gets its own
  CU-masked stream (``hipExtStreamCreateWithCUMask``), the per-queue form of
  ``ROC_GLOBAL_CU_MASK``, and its graph is captured under the slice-budgeted
  kernel configs a masked process pod uses (``ops.set_cu_budget``: grids
  sized to its CUs).  Unmasked tenants share every CU, which is MPS's
  default and the chart's default for pod-server nodes (cuPolicy auto).
* **Kernel configs.**  Tenants run the fractional-pod kernel configs of
  :func:`nos_amd.models.pod.kernel_config` while co-tenants fill the CU slots
  (no key splits, x6 GEMMs on 128x128 tiles).  A tenant alone on the GPU
  needs the whole-GPU configs instead (fewest rounds of tiles, attention key
  splits): configs are baked into a graph at capture, so an unmasked tenant
  gets a second, *solo* graph captured under the whole-GPU configs in the
  same memory pool (a tenant never replays two graphs at once), and a lane
  replays it when no other job is running or queued (``solo_graphs``).

``device="cpu"`` runs programs eagerly on the CPU, without streams or graphs
(protocol tests on machines without a GPU).
"""
from __future__ import annotations

import collections
import contextlib
import logging
import os
import socket
import threading
import time
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

from ..observability import metrics as M
from . import protocol as P

log = logging.getLogger("nos_amd.podserver")

DEFAULT_LANES = 16  # 28-tenant fleet with the h3 kernels: 16 > 12 > 8 > 20 (profiles/r04_h3_lanes_ab.json)
DEFAULT_MAX_TENANTS = 48  # MPS's client limit per server (Volta+)


@dataclass
class Tenant:
    id: int
    pod: str
    memory_limit_gb: float
    dtype: str
    model: object                  # the compiled program (program.CompiledProgram)
    x: object                      # static input tensor (graph input)
    stream: object = None          # own CU-masked stream (masked tenants), else None
    graph: object = None
    outputs: tuple = ()
    footprint_gb: float = 0.0
    cu_mask: str | None = None
    solo_graph: object = None      # whole-GPU configs, replayed when the tenant runs alone
    solo_outputs: tuple = ()
    completed: int = 0
    solo_completed: int = 0
    gpu_s: float = 0.0
    registered_at: float = field(default_factory=time.monotonic)
    token: str | None = None       # allocation token (None: open admission)
    record_path: object = None     # the device plugin's allocation record
    device_ids: tuple = ()
    conn: object = None            # the client connection (closed on eviction)
    program: str = ""
    compile_stats: dict = field(default_factory=dict)
    evicted: str | None = None
    id_bound: int | None = None    # token-id input: ids must lie in [0, id_bound)
    alts: dict = field(default_factory=dict)   # other input shapes -> _Variant (same weights)
    trainer: object = None         # a training tenant (training.Trainer): steps instead of inferences
    latency: bool = False          # served by the priority lanes (a generation step per request)
    state: dict = field(default_factory=dict)       # persistent buffers (K / V caches, positions), every variant's
    pos_limits: dict = field(default_factory=dict)  # position state -> rows of the caches written at it
    host: dict = field(default_factory=dict)        # pinned staging buffers (input, outputs, counters)


@dataclass
class _Variant:
    """One more input shape of a tenant (program.parse_variants): its own
    compiled program, static input and graphs over the tenant's weights."""
    model: object
    x: object
    graph: object = None
    outputs: tuple = ()
    solo_graph: object = None
    solo_outputs: tuple = ()
    host: dict = field(default_factory=dict)


@dataclass
class _Job:
    tenant: Tenant
    payload: bytes
    want_outputs: bool | list     # True: every output; a list: those output indices
    shape: tuple | None = None
    kind: str = "infer"            # or "train": one optimisation step, payload = input + target
    x_bytes: int = 0
    steps: int = 1                 # "generate": runs, each fed the previous run's output ``feed``
    feed: int = -1
    loss: float | None = None
    done: threading.Event = field(default_factory=threading.Event)
    t_enq: float = field(default_factory=time.monotonic)
    t_start: float = 0.0
    t_end: float = 0.0
    outputs: list = field(default_factory=list)
    error: str | None = None
    state: dict | None = None      # the tenant's counters after the run (stateful tenants)


class AdmissionError(RuntimeError):
    pass


def _wire_dtype(x) -> str:
    """The element type a tenant's input travels as: "i32" (token ids) or "f32"."""
    return "i32" if str(getattr(x, "dtype", "")) == "torch.int32" else "f32"


def _pos_limits(progs) -> dict:
    """Position state -> the fewest cache rows any ``kv_write`` at it writes
    (past that the writes are dropped: the server reports the overflow)."""
    lim: dict[str, int] = {}
    for p in progs:
        for n in p.nodes:
            if n.op == "kv_write":
                root = p.state_root.get(n.inputs[2], n.inputs[2])
                rows = p.values[n.inputs[0]].shape[1]
                lim[root] = min(lim.get(root, rows), rows)
    return lim


def _target_wire(trainer) -> str:
    """A training tenant's target on the wire: class ids (i32) or values (f32)."""
    return "i32" if trainer.spec["target_dtype"] == "i32" else "f32"


def _check_wire_dtype(sent, want: str, what: str) -> None:
    """The payload carries no dtype of its own: a request that names one must
    name the tenant's (an int array read as float32 bit patterns, or floats
    read as ids, would run without error and answer garbage).  Requests of
    older clients name none and are taken as the tenant's type."""
    if sent is not None and sent != want:
        raise ValueError(f"{what} sent as {sent!r}, the tenant's model takes {want!r}")


def _host_array(o) -> np.ndarray:
    """An output on the host as fp32.  A row-strided output (a column slice of
    a merged GEMM's result, e.g. the class logits beside the box columns)
    travels as the covering row block and is sliced on the host -- no device
    copy kernel to make it contiguous first."""
    o = o.detach()
    block = _covering_block(o) if o.is_cuda else None
    if block is not None:
        return block.cpu()[:, :o.shape[-1]].float().reshape(o.shape).numpy()
    # to the host first, then fp32: a device-side cast (an int32 next-token id, a bf16
    # output) would be one more kernel per request on the lane
    return o.cpu().float().numpy()


def _covering_block(o):
    """The contiguous ``(rows, ld)`` block a row-strided output lies in
    (``o.view(-1, N)`` with unit column stride), or None."""
    import torch

    if o.is_contiguous() or o.dim() < 2 or o.stride(-1) != 1 or not o.numel():
        return None
    N = o.shape[-1]
    try:
        o2 = o.view(-1, N)
    except RuntimeError:
        return None
    rows, ld = o2.shape[0], o2.stride(0)
    if o2.storage_offset() + rows * ld > o2.untyped_storage().nbytes() // o2.element_size():
        return None
    return torch.as_strided(o2, (rows, ld), (ld, 1))


def _pinned(cache: dict, key, shape, dtype):
    """A pinned host staging buffer of ``shape`` / ``dtype``, kept in ``cache``
    (a tenant's or variant's): one per input / output slot, reused by every
    request (a tenant's requests run one at a time)."""
    import torch

    b = cache.get(key)
    if b is None or tuple(b.shape) != tuple(shape) or b.dtype != dtype:
        b = cache[key] = torch.empty(tuple(shape), dtype=dtype, pin_memory=True)
    return b


def _fetch_start(o, cache: dict, key):
    """Queue ``o``'s device -> host copy into a pinned buffer on the current
    stream and return the function that, once the stream is synchronised,
    gives it as fp32 numpy (what ``_host_array`` gives).  A decode step's
    outputs and counters then reach the host behind ONE synchronisation
    instead of a blocking pageable copy each."""
    import torch

    o = o.detach()
    if not o.is_cuda:
        return lambda: _host_array(o)
    block = _covering_block(o)
    src = block if block is not None else o
    if not src.is_contiguous():
        return lambda: _host_array(o)     # after the synchronisation: a plain blocking copy
    hb = _pinned(cache, key, src.shape, src.dtype)
    hb.copy_(src, non_blocking=True)

    def done():
        h = hb[:, :o.shape[-1]].reshape(o.shape) if block is not None else hb
        if h.dtype in (torch.bfloat16, torch.float16):
            h = h.float()
        return np.array(h.numpy(), dtype=np.float32)   # a copy: the buffer serves the next request

    return done


class _JobQueue:
    """The lanes' work queue: two FIFOs, latency requests before throughput
    ones.  ``get(hi_only=True)`` (a priority lane) waits for a latency
    request only, ``get(lo_only=True)`` (a throughput lane beside CU-reserved
    priority lanes) for a throughput one; ``close()`` makes every ``get``
    return None."""

    def __init__(self):
        self._cv = threading.Condition()
        self._hi: collections.deque = collections.deque()
        self._lo: collections.deque = collections.deque()
        self._closed = False

    def put(self, job, hi: bool = False) -> None:
        with self._cv:
            (self._hi if hi else self._lo).append(job)
            self._cv.notify_all()   # a priority lane may be the one waiting

    def get(self, hi_only: bool = False, lo_only: bool = False):
        with self._cv:
            while True:   # what was queued before close() still runs
                if self._hi and not lo_only:
                    return self._hi.popleft()
                if self._lo and not hi_only:
                    return self._lo.popleft()
                if self._closed:
                    return None
                self._cv.wait()

    def qsize(self) -> int:
        with self._cv:
            return len(self._hi) + len(self._lo)

    def close(self) -> None:
        with self._cv:
            self._closed = True
            self._cv.notify_all()


class PodServer:
    def __init__(self, socket_path: str | os.PathLike, device: str = "cuda", lanes: int = DEFAULT_LANES,
                 max_tenants: int = DEFAULT_MAX_TENANTS, memory_gb: float | None = None, graphs: bool = True,
                 kernel_config: dict | None = None, solo_graphs: bool = True,
                 allocations_dir: str | os.PathLike | None = None, pod_resources=None,
                 reap_interval_s: float = 1.0, max_inflight_register_gb: float = 16.0,
                 register_timeout_s: float = 30.0, register_min_mb_s: float = 50.0, priority_lanes: int = 0,
                 latency_cus: int = 0, masked_queues: int = 8):
        """``allocations_dir``: this GPU's allocation records (tokens
        required; allocations.py).  Without it admission is open: the client
        declares its slice, which must be > 0 when the server accounts
        memory (tests, bare metal).  ``pod_resources``: a PodResources lister
        (resource/client.py) -- tenants whose devices no pod holds any more
        are evicted.  ``register_timeout_s`` + payload / ``register_min_mb_s``:
        the deadline of a register payload once its header arrived (a stalled
        sender's claim is released and its connection closed).
        ``priority_lanes``: extra lanes on high-priority streams that serve
        only latency tenants (stateful decoders by default, or a register
        request with ``"priority": "latency"``); every lane takes a waiting
        latency request before any throughput request, so a generation step
        never queues behind throughput tenants' inferences.  ``latency_cus``
        (a multiple of 8, XCD-symmetric): that many CUs reserved for the
        priority lanes -- their streams are CU-masked to them and the other
        lanes' to the rest, so a decode step's chain of small kernels never
        waits for CUs held by a throughput tenant's long workgroups.
        ``masked_queues``: with ``latency_cus``, the number of CU-masked
        streams (each a hardware queue) the throughput lanes share."""
        if lanes < 1:
            raise ValueError("lanes must be >= 1")
        self.path = Path(socket_path)
        self.device = device
        self.gpu = device == "cuda"
        self.lanes_n = lanes
        self.max_tenants = max_tenants
        self.graphs = graphs and self.gpu
        self.tenants: dict[int, Tenant] = {}
        self._next_id = 1
        self._lock = threading.Lock()          # tenant table
        self._build_lock = threading.Lock()    # one registration (build + capture + accounting) at a time
        self._jobs = _JobQueue()   # latency tenants' requests dequeued first
        self.priority_lanes_n = max(0, int(priority_lanes))
        self.latency_cus = int(latency_cus)
        if self.latency_cus and (self.latency_cus % 8 or self.latency_cus < 0 or not self.priority_lanes_n):
            raise ValueError("latency_cus must be a positive multiple of 8 (one share per XCD) with priority lanes")
        self.masked_queues = int(masked_queues)
        if self.masked_queues < 1:
            raise ValueError("masked_queues must be >= 1")
        self._masked: list = []   # CU-masked lane streams (latency_cus) to close at stop
        self._hi_lanes: list = []
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self._conns: dict[socket.socket, threading.Thread] = {}  # open client connections
        self._lanes: list = []
        self._sock: socket.socket | None = None
        self.kernel_config = kernel_config
        self.solo_graphs = solo_graphs and self.graphs
        self.solo_config: dict | None = None
        self._busy = 0                          # lanes running a job
        self.memory_gb = memory_gb
        self.info: dict = {}
        self.gpu_label = os.environ.get("HIP_VISIBLE_DEVICES", "0") if self.gpu else "cpu"  # metrics label
        self.allocations_dir = Path(allocations_dir) if allocations_dir else None
        self.pod_resources = pod_resources
        self.reap_interval_s = reap_interval_s
        self._pending: dict[int, float] = {}    # tenant id -> slice GB reserved while its build runs
        self._tokens: set[str] = set()           # tokens holding a tenant (or a pending build)
        self._inflight_bytes = 0                 # register payload bytes claimed and not yet built
        self.max_inflight_register_bytes = int(max_inflight_register_gb * 2 ** 30)
        self.register_timeout_s = float(register_timeout_s)
        self.register_min_mb_s = float(register_min_mb_s)
        self.evictions = 0

    # ------------------------------------------------------------ lifecycle
    def _init_device(self) -> None:
        import torch

        if not self.gpu:
            torch.set_num_threads(1)
            self.info = {"device": "cpu", "lanes": self.lanes_n}
            return
        from ..models.pod import kernel_config
        from ..ops import _lib

        _lib.require_native_on_gpu()
        torch.cuda.set_device(0)
        torch.backends.cuda.matmul.allow_tf32 = False
        # fractional-pod configs: the co-tenants fill the CU slots (pod.kernel_config)
        cfg = self.kernel_config or kernel_config(0.5, os.environ, 0)
        self.kernel_config = cfg
        if self.solo_graphs:
            solo = kernel_config(1.0, os.environ, 0)
            self.solo_config = solo if solo != cfg else None
        self._apply_config(cfg)
        props = torch.cuda.get_device_properties(0)
        total_gb = props.total_memory / 2 ** 30
        self.memory_gb = min(self.memory_gb or total_gb, total_gb)
        # lanes first: with GPU_MAX_HW_QUEUES >= lanes each gets its own HW queue
        if self.latency_cus:
            # CU mask bit i sits on XCD i mod 8: CUs 0 .. n-1 are n / 8 per XCD
            from ..ops.streams import CUMaskedStream

            ncu = props.multi_processor_count
            if self.latency_cus >= ncu:
                raise ValueError(f"latency_cus {self.latency_cus} leaves no CU of {ncu} to the other lanes")
            rest = range(self.latency_cus, ncu)
            # every CU-masked stream is a hardware queue of its own (GPU_MAX_HW_QUEUES does not
            # pool them): past ~10 of them the decoders starved (16 + 2: 182 ms / token, 8 + 2:
            # 5 ms), so the throughput lanes share at most masked_queues of them, round robin
            nq = min(self.lanes_n, self.masked_queues)
            self._masked = [CUMaskedStream(rest, ncu) for _ in range(nq)]
            self._masked += [CUMaskedStream(range(self.latency_cus), ncu) for _ in range(self.priority_lanes_n)]
            self._lanes = [self._masked[i % nq].torch for i in range(self.lanes_n)]
            self._hi_lanes = [m.torch for m in self._masked[nq:]]
        else:
            self._lanes = [torch.cuda.Stream() for _ in range(self.lanes_n)]
            # latency lanes: the highest stream priority (HSA queue priority), dispatched first
            hi = torch.cuda.Stream.priority_range()[1] if hasattr(torch.cuda.Stream, "priority_range") else -1
            self._hi_lanes = [torch.cuda.Stream(priority=hi) for _ in range(self.priority_lanes_n)]
        self._setup_stream = torch.cuda.Stream()
        self.info = {"device": props.name, "multiprocessor_count": props.multi_processor_count,
                     "lanes": self.lanes_n, "priority_lanes": self.priority_lanes_n, "latency_cus": self.latency_cus,
                     "masked_queues": min(self.lanes_n, self.masked_queues) if self.latency_cus else 0,
                     "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                     "memory_gb": round(self.memory_gb, 1), "kernel_config": cfg,
                     "solo_kernel_config": self.solo_config,
                     "hip_visible_devices": os.environ.get("HIP_VISIBLE_DEVICES")}

    @staticmethod
    def _apply_config(cfg: dict) -> None:
        """Process-wide kernel configs; a graph keeps the ones it was captured under."""
        from ..ops import set_attention_f32_variant, set_f32_math, set_gemm_f32_policy, set_gemm_f32x6_tile, \
            set_gemm_f32h3_hot_bn, set_gemm_f32h3_hot_ring, set_gemm_f32h3_layout, set_gemm_f32h3_lds_epilogue, \
            set_gemm_f32h3_lna_wide, set_gemm_policy, set_ln_handoff

        set_gemm_policy(cfg["gemm_bf16"])
        set_gemm_f32_policy(cfg["gemm_f32"])
        set_attention_f32_variant(cfg["attention_f32"])
        set_f32_math(cfg["f32_math"])
        set_gemm_f32x6_tile(cfg["gemm_f32x6_tile"])
        set_ln_handoff(cfg.get("ln_handoff", "on") == "on")
        set_gemm_f32h3_lds_epilogue(cfg.get("h3_epilogue", "lds") == "lds")
        set_gemm_f32h3_layout(cfg.get("h3_layout", "2x2"))
        set_gemm_f32h3_hot_ring(int(cfg.get("h3_hot_ring", "2")))
        set_gemm_f32h3_hot_bn(int(cfg.get("h3_hot_bn", "128")))
        set_gemm_f32h3_lna_wide(cfg.get("h3_lna_wide", "off") == "on")

    def start(self) -> "PodServer":
        self._init_device()
        self.path.parent.mkdir(parents=True, exist_ok=True)
        if self.path.exists():
            self.path.unlink()
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        tmp = self.path.with_name(self.path.name + ".tmp")
        if tmp.exists():
            tmp.unlink()
        s.bind(str(tmp))
        s.listen(256)
        os.replace(tmp, self.path)  # the socket appears only once the server accepts
        self._sock = s
        for i in range(self.lanes_n):
            t = threading.Thread(target=self._lane, args=(i,), name=f"lane-{i}", daemon=True)
            t.start()
            self._threads.append(t)
        for i in range(self.priority_lanes_n):
            t = threading.Thread(target=self._lane, args=(i, True), name=f"hi-lane-{i}", daemon=True)
            t.start()
            self._threads.append(t)
        t = threading.Thread(target=self._accept, name="accept", daemon=True)
        t.start()
        self._threads.append(t)
        if self.allocations_dir is not None or self.pod_resources is not None:
            t = threading.Thread(target=self._reap, name="reaper", daemon=True)
            t.start()
            self._threads.append(t)
        log.info("pod server on %s: %s", self.path, self.info)
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._sock is not None:
            try:
                self._sock.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
            self._sock.close()
        # close every client connection and wait for its thread: each one
        # unregisters (frees) its tenant, so no thread touches the GPU once stop()
        # returns -- a daemon thread still freeing a HIP graph while the
        # interpreter exits aborts the process
        with self._lock:
            conns = list(self._conns.items())
        for c, _ in conns:
            try:
                c.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
        for _, t in conns:
            t.join(timeout=30)
        self._jobs.close()
        for t in self._threads:
            t.join(timeout=10)
        with self._lock:
            left = list(self.tenants.values())
            self.tenants.clear()
        for t in left:
            self._free(t)
        try:
            self.path.unlink()
        except FileNotFoundError:
            pass
        if self.gpu:
            import torch

            torch.cuda.synchronize()
            for m in self._masked:
                m.close()
            self._masked = []

    def serve_forever(self) -> None:
        while not self._stop.is_set():
            self._stop.wait(1.0)

    # ------------------------------------------------------------ connections
    def _accept(self) -> None:
        while not self._stop.is_set():
            try:
                conn, _ = self._sock.accept()
            except OSError:
                return
            t = threading.Thread(target=self._serve, args=(conn,), daemon=True)
            with self._lock:
                self._conns[conn] = t
            t.start()

    def _serve(self, conn: socket.socket) -> None:
        tenant: Tenant | None = None
        claim: dict = {}   # this connection's register reservation (_claim), made before its payload is read

        def limit(req: dict, npay: int) -> int:
            if req.get("op") != "register":
                return P.MAX_PAYLOAD
            claim.clear()
            if tenant is not None:
                claim["error"] = "AdmissionError: connection already holds a tenant"
                return 0
            try:
                return self._claim(req, npay, claim)
            except (AdmissionError, TypeError, ValueError) as e:  # bad field types are a refusal, not a crash
                claim.clear()
                claim["error"] = f"AdmissionError: {e}"
                return 0

        def deadline(req: dict, npay: int) -> float | None:
            # only a claimed register payload holds a reservation worth bounding
            if req.get("op") != "register" or not claim.get("pending"):
                return None
            return self.register_timeout_s + npay / (self.register_min_mb_s * 1e6)

        try:
            while not self._stop.is_set():
                try:
                    req, payload = P.recv_msg(conn, limit, deadline)
                except P.ProtocolError as e:  # payload drained: the connection is still in step
                    err = claim.pop("error", None) or f"{type(e).__name__}: {e}"
                    self._release_claim(claim)
                    P.send_msg(conn, {"ok": False, "error": err})
                    continue
                except (ConnectionError, OSError, ValueError):
                    self._release_claim(claim)
                    return
                op = req.get("op")
                try:
                    if op == "register":
                        if "error" in claim:
                            raise AdmissionError(claim.pop("error").split(": ", 1)[-1])
                        tenant = self._register(req, payload, conn, claim)
                        P.send_msg(conn, {"ok": True, "tenant": tenant.id, "footprint_gb": tenant.footprint_gb,
                                          "memory_limit_gb": tenant.memory_limit_gb, "cu_mask": tenant.cu_mask,
                                          "input_shape": list(tenant.x.shape),
                                          "input_dtype": _wire_dtype(tenant.x),
                                          "target_dtype": (_target_wire(tenant.trainer)
                                                           if tenant.trainer is not None else None),
                                          "input_shapes": [list(tenant.x.shape)] + [list(k) for k in tenant.alts],
                                          "server": self.info,
                                          "program": tenant.program, "compile": tenant.compile_stats,
                                          "tenants": len(self.tenants)})
                    elif op == "infer":
                        if tenant is None:
                            raise AdmissionError("register first")
                        shp = req.get("shape")
                        shp = tuple(int(d) for d in shp) if isinstance(shp, list) and len(shp) <= 8 else None
                        _check_wire_dtype(req.get("dtype"), _wire_dtype(tenant.x), "input")
                        want = req.get("outputs")
                        if isinstance(want, list):   # a selection of the program's outputs, by index
                            if not all(isinstance(i, int) and not isinstance(i, bool) for i in want) or len(want) > 64:
                                raise ValueError("outputs must be true / false or a list of output indices")
                        else:
                            want = bool(want)
                        job = _Job(tenant, payload, want, shp)
                        self._jobs.put(job, hi=tenant.latency)
                        job.done.wait()
                        if job.error:
                            raise RuntimeError(job.error)
                        descs, out = P.pack_arrays(job.outputs) if job.outputs else ([], b"")
                        rep = {"ok": True, "queue_us": round(1e6 * (job.t_start - job.t_enq), 1),
                               "gpu_us": round(1e6 * (job.t_end - job.t_start), 1), "outputs": descs}
                        if job.state is not None:
                            rep["state"] = job.state
                        P.send_msg(conn, rep, out)
                    elif op == "generate":   # a stateful tenant's decode loop, run in the server
                        if tenant is None:
                            raise AdmissionError("register first")
                        if not tenant.state or tenant.trainer is not None:
                            raise ValueError("generate needs a stateful (decode) tenant")
                        n, feed = req.get("steps"), req.get("output", -1)
                        if (not isinstance(n, int) or isinstance(n, bool) or not 1 <= n <= 4096
                                or not isinstance(feed, int) or isinstance(feed, bool)):
                            raise ValueError("generate: steps must be an int in [1, 4096], output an output index")
                        shp = req.get("shape")
                        shp = tuple(int(d) for d in shp) if isinstance(shp, list) and len(shp) <= 8 else None
                        _check_wire_dtype(req.get("dtype"), _wire_dtype(tenant.x), "input")
                        job = _Job(tenant, payload, [feed], shp, kind="generate", steps=n, feed=feed)
                        self._jobs.put(job, hi=tenant.latency)
                        job.done.wait()
                        if job.error:
                            raise RuntimeError(job.error)
                        descs, out = P.pack_arrays(job.outputs)
                        P.send_msg(conn, {"ok": True, "queue_us": round(1e6 * (job.t_start - job.t_enq), 1),
                                          "gpu_us": round(1e6 * (job.t_end - job.t_start), 1), "outputs": descs,
                                          "state": job.state}, out)
                    elif op == "reset":
                        if tenant is None:
                            raise AdmissionError("register first")
                        self._reset_state(tenant)
                        P.send_msg(conn, {"ok": True, "state": self._counters(tenant)})
                    elif op == "train":
                        if tenant is None or tenant.trainer is None:
                            raise AdmissionError("train needs a training tenant (register with a train spec)")
                        xb = req.get("x_bytes")
                        if not isinstance(xb, int) or not 0 <= xb <= len(payload):
                            raise ValueError("train: x_bytes must split the payload into input + target")
                        _check_wire_dtype(req.get("dtype"), _wire_dtype(tenant.trainer.x), "input")
                        _check_wire_dtype(req.get("target_dtype"), _target_wire(tenant.trainer), "target")
                        job = _Job(tenant, payload, False, kind="train", x_bytes=xb)
                        self._jobs.put(job)
                        job.done.wait()
                        if job.error:
                            raise RuntimeError(job.error)
                        P.send_msg(conn, {"ok": True, "loss": job.loss, "step": tenant.trainer.steps,
                                          "queue_us": round(1e6 * (job.t_start - job.t_enq), 1),
                                          "gpu_us": round(1e6 * (job.t_end - job.t_start), 1)})
                    elif op == "weights":
                        if tenant is None or tenant.trainer is None:
                            raise AdmissionError("weights: only a training tenant's weights change")
                        P.send_msg(conn, {"ok": True, "step": tenant.trainer.steps}, tenant.trainer.weights_bytes())
                    elif op == "checkpoint":
                        if tenant is None or tenant.trainer is None:
                            raise AdmissionError("checkpoint: only a training tenant has optimizer state")
                        P.send_msg(conn, {"ok": True, "step": tenant.trainer.steps},
                                   tenant.trainer.checkpoint_bytes())
                    elif op == "stats":
                        P.send_msg(conn, {"ok": True, **self.stats()})
                    elif op == "close":
                        if tenant is not None:  # freed before the ack: close() returns with the slice released
                            self._unregister(tenant)
                            tenant = None
                        P.send_msg(conn, {"ok": True})
                        return
                    else:
                        raise P.ProtocolError(f"unknown op {op!r}")
                except Exception as e:  # noqa: BLE001 -- reported to this client; the server keeps serving
                    if op == "register":
                        self._release_claim(claim)
                    P.send_msg(conn, {"ok": False, "error": f"{type(e).__name__}: {e}"})
        finally:
            self._release_claim(claim)
            if tenant is not None:
                self._unregister(tenant)
            with self._lock:
                self._conns.pop(conn, None)
            conn.close()

    def _claim(self, req: dict, npay: int, claim: dict) -> int:
        """Admit a register request BEFORE its payload is read: check the
        token, claim it (one tenant per token), reserve a tenant slot, the
        slice's memory and ``npay`` bytes of the server's in-flight register
        budget, all under the lock.  Returns the payload limit (the slice:
        weights may fill it, the static estimate then checks weights +
        activations).  A second register with the same token, or many
        connections sending slice-sized weights at once, are refused before
        any of their bytes are buffered in host memory."""
        limit, mask, token, record, dev_ids = self._admission(req)
        cap = int(limit * 2 ** 30) if limit else int((self.memory_gb or 64) * 2 ** 30)
        with self._lock:
            if token is not None and token in self._tokens:
                raise AdmissionError("the allocation already holds a tenant (or a registration in flight)")
            if len(self.tenants) + len(self._pending) >= self.max_tenants:
                raise AdmissionError(f"server full ({self.max_tenants} tenants)")
            if self.memory_gb and limit:
                held = sum(t.memory_limit_gb for t in self.tenants.values()) + sum(self._pending.values())
                if held + limit > self.memory_gb + 1e-6:
                    raise AdmissionError(f"slice of {limit} GB does not fit: {held} of {self.memory_gb} GB held")
            # host memory: registrations buffer their weights here; one may always
            # proceed (a big tenant is never starved), more only within the budget
            if self._inflight_bytes and self._inflight_bytes + min(npay, cap) > self.max_inflight_register_bytes:
                raise AdmissionError(f"{self._inflight_bytes / 2 ** 30:.1f} GB of registrations in flight; retry")
            tid = self._next_id
            self._next_id += 1
            self._pending[tid] = limit
            if token is not None:
                self._tokens.add(token)
            nb = min(npay, cap)
            self._inflight_bytes += nb
        claim.update(tid=tid, limit=limit, mask=mask, token=token, record=record, dev_ids=dev_ids, nbytes=nb,
                     pending=True)
        return cap

    def _release_claim(self, claim: dict, keep_token: bool = False) -> None:
        """Undo :meth:`_claim` (idempotent): the pending slot and memory, the
        in-flight bytes and, unless the tenant now holds it, the token."""
        if not claim.get("pending"):
            return
        with self._lock:
            self._pending.pop(claim["tid"], None)
            self._inflight_bytes -= claim["nbytes"]
            if claim["token"] is not None and not keep_token:
                self._tokens.discard(claim["token"])
        claim.clear()

    # ------------------------------------------------------------ tenants
    def _admission(self, req: dict) -> tuple[float, str | None, str | None, object, tuple]:
        """(slice GB, CU mask, token, record path, device ids) of a register
        request: from the device plugin's record when the server has an
        allocations directory, else as the client declares them."""
        if self.allocations_dir is not None:
            from .allocations import lookup

            token = req.get("token")
            if not token:
                raise AdmissionError("no allocation token: this pod was not allocated a pod-server slice "
                                     "(NOS_AMD_POD_TOKEN)")
            hit = lookup(self.allocations_dir, str(token))
            if hit is None:
                raise AdmissionError("unknown allocation token (not allocated on this GPU, or released)")
            rec, path = hit
            limit = float(rec.get("memory_gb") or 0)
            if limit <= 0:
                raise AdmissionError("the allocation carries no memory slice")
            return limit, rec.get("cu_mask") or None, str(token), path, tuple(rec.get("device_ids", ()))
        limit = float(req.get("memory_limit_gb") or 0)
        if self.memory_gb and limit <= 0:
            raise AdmissionError("a memory slice (memory_limit_gb > 0) is required: the server accounts memory")
        return limit, req.get("cu_mask") or None, None, None, ()

    def _register(self, req: dict, payload: bytes = b"", conn=None, claim: dict | None = None) -> Tenant:
        """Build a tenant for a register request whose slot, memory and token
        :meth:`_claim` reserved before its payload was read (direct callers
        without a claim get one here); the claim is released on failure."""
        from . import program as PG

        if claim is None or not claim.get("pending"):
            claim = {}
            self._claim(req, len(payload), claim)
        try:
            if "program" not in req:
                raise AdmissionError("register carries no program (nos-amd.program/v1 op graph + weights)")
            if req.get("priority") not in (None, "latency", "throughput"):
                raise AdmissionError("priority must be 'latency' or 'throughput'")
            extra = req.get("variants") or []
            if not isinstance(extra, list):
                raise AdmissionError("variants must be a list of programs")
            limit, mask, tid = claim["limit"], claim["mask"], claim["tid"]
            if req.get("train") is not None:
                from .training import parse_train_spec, train_bytes_estimate

                if extra:
                    raise AdmissionError("a training tenant takes one input shape (no variants)")
                prog = PG.parse(req["program"], payload)
                if prog.state:
                    raise AdmissionError("a stateful program (K / V caches) cannot be a training tenant")
                spec = parse_train_spec(req["train"], prog)
                need = train_bytes_estimate(prog, spec) / 2 ** 30
                if limit and need > limit:
                    raise AdmissionError(f"training tenant needs {need:.2f} GB (static estimate), "
                                         f"its slice has {limit} GB")
                state = None
                if spec["resume"]:   # payload = weights + optimizer state (Trainer.checkpoint_bytes)
                    from .training import state_nbytes

                    wlen = max((o + n for o, n in prog.param_layout.values()), default=0)
                    if len(payload) != wlen + state_nbytes(prog, spec):
                        raise AdmissionError(f"resume payload of {len(payload)} bytes: the weights take {wlen}, "
                                             f"the optimizer state {state_nbytes(prog, spec)}")
                    state = bytes(payload[wlen:])
                with self._build_lock:
                    t = self._build_trainer(tid, req, prog, spec, limit, mask, state)
                progs = None
            else:
                progs = PG.parse_variants([req["program"], *extra], payload, gpu=self.gpu)
            if progs is not None:
                # the weights once, every variant's activations, planes and folded copies
                need = sum(p.bytes_estimate_for(self.kernel_config) for p in progs) / 2 ** 30
                need -= (len(progs) - 1) * (progs[0].param_bytes + progs[0].state_bytes) / 2 ** 30
                if limit and need > limit:
                    raise AdmissionError(f"tenant needs {need:.2f} GB (static estimate), its slice has {limit} GB")
                with self._build_lock:
                    t = self._build(tid, req, progs, limit, mask)
        except BaseException:
            self._release_claim(claim)
            raise
        t.token, t.record_path, t.device_ids, t.conn = claim["token"], claim["record"], claim["dev_ids"], conn
        prio = req.get("priority")
        # a stateful tenant (a decoder generating token by token) is a latency tenant unless it says otherwise
        t.latency = prio == "latency" or (prio is None and bool(t.state))
        with self._lock:
            self.tenants[tid] = t
            M.PODSERVER_TENANTS.labels(self.gpu_label).set(len(self.tenants))
        self._release_claim(claim, keep_token=True)
        log.info("tenant %d (%s, %s) registered: %.3f GB of a %s GB slice", tid, t.pod, t.program, t.footprint_gb,
                 limit or "-")
        return t

    def _build(self, tid: int, req: dict, progs, limit: float, mask: str | None) -> Tenant:
        """Compile and capture a tenant: one program per input shape
        (``progs[0]`` the primary; or one Program), all over one set of
        weight tensors."""
        import torch

        from ..models.yolos import GraphedTenant

        progs = progs if isinstance(progs, list) else [progs]
        pod = str(req.get("pod", tid))[:253]
        prog = progs[0]
        dtype = prog.inputs[0].dtype
        if not self.gpu:
            with torch.no_grad():
                params = prog.tensors("cpu")
                state = prog.state_tensors("cpu")
                derived: dict = {}
                built = [(p.compile("cpu", params=params, state=state, derived=derived), p.input_tensor("cpu"))
                         for p in progs]
                del derived
            m, x = built[0]
            return Tenant(tid, pod, limit, dtype, m, x, program=prog.name, compile_stats=dict(m.stats), cu_mask=mask,
                          id_bound=prog.id_bound(), alts={tuple(xv.shape): _Variant(mv, xv) for mv, xv in built[1:]},
                          state=state, pos_limits=_pos_limits(progs))
        base = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        stream = None
        t0 = time.monotonic()
        times = {}
        try:
            with torch.no_grad(), torch.cuda.stream(self._setup_stream):
                params = prog.tensors("cuda")
                state = prog.state_tensors("cuda")   # allocated once: a replay never grows it
                derived: dict = {}   # folded / merged weights: one copy for all the variants
                built = [(p.compile("cuda", params=params, state=state, derived=derived), p.input_tensor("cuda"))
                         for p in progs]
                del params, derived   # each compiled program holds the weights it reads
            self._setup_stream.synchronize()
            times["compile_ms"] = round(1e3 * (time.monotonic() - t0), 1)
            budget_cfg = None
            if mask:
                from ..bench_support import cus_from_hex
                from ..models.pod import kernel_config
                from ..ops.streams import CUMaskedStream

                cus = cus_from_hex(mask)
                stream = CUMaskedStream(cus, self.info["multiprocessor_count"])
                # a CU-mask slice plans for its own CUs: slice-sized persistent
                # grids and the budget-aware configs a masked process pod uses
                frac = limit / self.memory_gb if limit and self.memory_gb else 0.5
                budget_cfg = (kernel_config(frac, os.environ, len(cus)), len(cus))
            variants = [self._capture(m, x, stream, budget_cfg, mask, GraphedTenant) for m, x in built]
            if state:   # the capture's warm-up runs advanced the state: a fresh sequence at position 0
                with torch.cuda.stream(self._setup_stream):
                    for st in state.values():
                        st.zero_()
                self._setup_stream.synchronize()
            peak = (torch.cuda.max_memory_allocated() - base) / 2 ** 30
            times["build_ms"] = round(1e3 * (time.monotonic() - t0), 1)
        except Exception:
            if stream is not None:
                stream.close()
            torch.cuda.empty_cache()
            raise
        v0 = variants[0]
        t = Tenant(tid, pod, limit, dtype, v0.model, v0.x, stream=stream, graph=v0.graph,
                   outputs=v0.outputs, footprint_gb=round(peak, 3), cu_mask=mask,
                   solo_graph=v0.solo_graph, solo_outputs=v0.solo_outputs,
                   program=prog.name, compile_stats={**v0.model.stats, **times}, id_bound=prog.id_bound(),
                   alts={tuple(v.x.shape): v for v in variants[1:]}, state=state, pos_limits=_pos_limits(progs))
        if limit and peak > limit:
            self._free(t)
            raise AdmissionError(f"tenant needs {peak:.2f} GB, its slice has {limit} GB")
        return t

    def _build_trainer(self, tid: int, req: dict, prog, spec: dict, limit: float, mask: str | None,
                       state: bytes | None = None) -> Tenant:
        """A training tenant (training.py): fp32 master weights, optimizer
        state and, on the GPU, forward + backward + step captured into one
        graph on the tenant's (CU-masked) stream."""
        import torch

        from .training import Trainer

        pod = str(req.get("pod", tid))[:253]
        if not self.gpu:
            tr = Trainer(prog, spec, "cpu", state)
            return Tenant(tid, pod, limit, "fp32", tr.module, tr.x, program=prog.name, cu_mask=mask, trainer=tr,
                          compile_stats={"train": spec["optimizer"], "loss": spec["loss"]},
                          id_bound=prog.id_bound())
        base = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        stream = None
        t0 = time.monotonic()
        try:
            if mask:
                from ..bench_support import cus_from_hex
                from ..ops.streams import CUMaskedStream

                stream = CUMaskedStream(cus_from_hex(mask), self.info["multiprocessor_count"])
            cap = stream.torch if stream else self._setup_stream
            with torch.cuda.stream(cap):
                tr = Trainer(prog, spec, "cuda", state)
            cap.synchronize()
            if self.graphs:
                tr.capture(cap)
            peak = (torch.cuda.max_memory_allocated() - base) / 2 ** 30
        except Exception:
            if stream is not None:
                stream.close()
            torch.cuda.empty_cache()
            raise
        t = Tenant(tid, pod, limit, "fp32", tr.module, tr.x, stream=stream, footprint_gb=round(peak, 3),
                   cu_mask=mask, program=prog.name, trainer=tr, id_bound=prog.id_bound(),
                   compile_stats={"train": spec["optimizer"], "loss": spec["loss"], "graph": tr.graph is not None,
                                  "build_ms": round(1e3 * (time.monotonic() - t0), 1)})
        if limit and peak > limit:
            self._free(t)
            raise AdmissionError(f"training tenant needs {peak:.2f} GB, its slice has {limit} GB")
        return t

    def _capture(self, m, x, stream, budget_cfg, mask, GraphedTenant) -> _Variant:
        """The graphs of one compiled program: under the slice's configs on
        its CU-masked stream, plus (unmasked) the whole-GPU solo graph in the
        same memory pool."""
        import torch

        gt = GraphedTenant(m, stream.torch if stream else self._setup_stream, x)
        with torch.no_grad():
            try:
                if budget_cfg is not None:
                    from ..ops import set_cu_budget

                    self._apply_config(budget_cfg[0])
                    set_cu_budget(budget_cfg[1])
                if self.graphs:  # the lanes keep replaying other tenants meanwhile
                    gt.capture(warmup=1, capture_error_mode="thread_local", light=True)
                else:
                    gt.launch()
                    gt.stream.synchronize()
            finally:
                if budget_cfg is not None:
                    set_cu_budget(0)
                    self._apply_config(self.kernel_config)
            solo = None
            if self.solo_config is not None and not mask and self.graphs:
                # the lanes only replay graphs, so switching the process-wide
                # configs for this capture changes no other tenant's kernels
                solo = GraphedTenant(m, self._setup_stream, x)
                try:
                    self._apply_config(self.solo_config)
                    # one warm-up: the first capture's already ran every kernel
                    solo.capture(warmup=1, capture_error_mode="thread_local", pool=gt.graph.pool(), light=True)
                finally:
                    self._apply_config(self.kernel_config)
        return _Variant(m, x, gt.graph, gt.outputs, solo.graph if solo else None, solo.outputs if solo else ())

    # ------------------------------------------------------------ eviction
    def evict(self, t: Tenant, reason: str) -> None:
        """Drop a tenant whose allocation is gone: close its connection (its
        thread unregisters and frees it once an in-flight replay finished)."""
        if t.evicted:
            return
        t.evicted = reason
        self.evictions += 1
        log.warning("evicting tenant %d (%s): %s", t.id, t.pod, reason)
        c = t.conn
        if c is not None:
            try:
                c.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass

    def reap_once(self) -> int:
        """Evict tenants whose allocation record vanished or whose devices no
        pod holds (PodResources).  Returns the number evicted."""
        with self._lock:
            ts = [t for t in self.tenants.values() if not t.evicted]
        used = None
        if self.pod_resources is not None:
            try:
                used = {d for pr in self.pod_resources.list() for c in pr.containers for cd in c.devices
                        for d in cd.device_ids}
            except Exception as e:  # kubelet unreachable: decide on the records alone
                log.info("PodResources unavailable: %s", e)
        n = 0
        for t in ts:
            if t.record_path is not None and not Path(t.record_path).exists():
                self.evict(t, "allocation released (record removed by the device plugin)")
                n += 1
            elif used is not None and t.device_ids and not any(d in used for d in t.device_ids):
                self.evict(t, "allocation released (no pod holds its devices in PodResources)")
                n += 1
        return n

    def _reap(self) -> None:
        while not self._stop.wait(self.reap_interval_s):
            try:
                self.reap_once()
            except Exception:
                log.exception("reaper pass failed")

    def _free(self, t: Tenant) -> None:
        t.graph = t.solo_graph = t.model = t.x = None
        t.outputs = t.solo_outputs = ()
        t.alts = {}
        t.trainer = None
        t.state = {}
        if t.stream is not None:
            t.stream.close()
            t.stream = None
        if self.gpu:
            import torch

            torch.cuda.empty_cache()

    def _unregister(self, t: Tenant) -> None:
        with self._lock:
            self.tenants.pop(t.id, None)
            if t.token is not None:
                self._tokens.discard(t.token)
            M.PODSERVER_TENANTS.labels(self.gpu_label).set(len(self.tenants))
        try:
            M.PODSERVER_INFERENCES.remove(self.gpu_label, t.pod)
        except KeyError:
            pass
        with self._build_lock:
            self._free(t)
        log.info("tenant %d (%s) left after %d inferences", t.id, t.pod, t.completed)

    def stats(self) -> dict:
        with self._lock:
            ts = [{"tenant": t.id, "pod": t.pod, "program": t.program, "completed": t.completed,
                   "solo_completed": t.solo_completed, "gpu_s": round(t.gpu_s, 4),
                   "footprint_gb": t.footprint_gb, "memory_limit_gb": t.memory_limit_gb, "cu_mask": t.cu_mask,
                   "kind": "train" if t.trainer is not None else "infer", "latency": t.latency,
                   "train_steps": t.trainer.steps if t.trainer is not None else 0}
                  for t in self.tenants.values()]
            pending = len(self._pending)
        return {"tenants": ts, "pending": pending, "server": self.info, "queued": self._jobs.qsize(), "pid": os.getpid(),
                "evictions": self.evictions}

    # ------------------------------------------------------------ lanes
    def _lane(self, i: int, hi: bool = False) -> None:
        import torch

        lane = (self._hi_lanes if hi else self._lanes)[i] if self.gpu else None
        while True:
            # beside CU-reserved priority lanes the throughput lanes leave latency requests
            # to them: a decode step queued on a shared masked stream behind an inference
            # waited for it (16 lanes over 8 masked queues: 12 ms / token)
            job = self._jobs.get(hi_only=hi, lo_only=not hi and bool(self.latency_cus))
            if job is None:
                return
            job.t_start = time.monotonic()
            with self._lock:
                self._busy += 1
                # no other tenant running or waiting
                alone = self._busy == 1 and self._jobs.qsize() == 0
            try:
                self._run(job, lane, alone)
            except Exception as e:  # reported to that tenant only
                job.error = f"{type(e).__name__}: {e}"
            finally:
                with self._lock:
                    self._busy -= 1
            job.t_end = time.monotonic()
            t = job.tenant
            t.completed += 1
            t.gpu_s += job.t_end - job.t_start
            M.PODSERVER_INFERENCES.labels(self.gpu_label, t.pod).inc()
            M.PODSERVER_REQUEST_TIME.labels(self.gpu_label).observe(job.t_end - job.t_enq)
            M.PODSERVER_QUEUED.labels(self.gpu_label).set(self._jobs.qsize())
            job.done.set()

    def _run(self, job: _Job, lane, alone: bool = False) -> None:
        import torch

        t = job.tenant
        if t.trainer is not None:
            return self._run_trainer(job, lane)
        # the primary shape, or the variant the request's input shape names
        # (an input of another shape but exactly one variant's size -- a
        # flattened array -- goes to that variant)
        v = t
        if t.alts and job.shape is not None and job.shape != tuple(t.x.shape):
            v = t.alts.get(job.shape)
            if v is None:
                n = len(job.payload) // 4
                fit = [w for w in (t, *t.alts.values()) if w.x.numel() == n]
                if len(fit) != 1:
                    raise ValueError(f"no program variant takes the input shape {list(job.shape)} "
                                     f"(registered: {[list(t.x.shape)] + [list(k) for k in t.alts]})")
                v = fit[0]
        x_in = None
        if job.payload:
            ids = str(v.x.dtype) == "torch.int32"
            x_in = np.frombuffer(job.payload, dtype=np.int32 if ids else np.float32)
            if x_in.size != v.x.numel():
                raise ValueError(f"input has {x_in.size} values, the tenant's model takes {v.x.numel()}")
            if ids and t.id_bound is not None and x_in.size and (x_in.min() < 0 or x_in.max() >= t.id_bound):
                raise ValueError(f"token ids must lie in [0, {t.id_bound})")
        gen = job.kind == "generate"

        def fed(outs) -> object:
            """generate: the output fed back as the next run's input (ids)."""
            if not -len(outs) <= job.feed < len(outs):
                raise ValueError(f"generate: output {job.feed} of {len(outs)}")
            o = outs[job.feed]
            if o.numel() != v.x.numel() or o.dtype != v.x.dtype:
                raise ValueError(f"generate: output {job.feed} {tuple(o.shape)} {o.dtype} does not feed the input "
                                 f"{tuple(v.x.shape)} {v.x.dtype}")
            return o

        with torch.no_grad():
            if not self.gpu:
                if x_in is not None:
                    v.x.copy_(torch.from_numpy(x_in.copy()).view(v.x.shape))
                v.outputs = outs = v.model(v.x)
                if gen:
                    toks = [fed(outs).clone()]
                    for _ in range(job.steps - 1):
                        v.x.copy_(toks[-1].reshape(v.x.shape))
                        v.outputs = outs = v.model(v.x)
                        toks.append(fed(outs).clone())
                    outs = [torch.stack(toks)]
                    job.want_outputs = [0]
                fetch = [lambda o=o: _host_array(o) for o in self._selected(outs, job.want_outputs)]
                counters = lambda: self._counters(t)  # noqa: E731
            else:
                s = t.stream.torch if t.stream is not None else lane
                with torch.cuda.stream(s):
                    if x_in is not None:
                        if str(v.x.dtype)[6:] == str(x_in.dtype):
                            # through a pinned buffer: an in-stream copy, no blocking pageable one
                            hb = _pinned(v.host, "x", v.x.shape, v.x.dtype)
                            hb.numpy().reshape(-1)[:] = x_in
                            v.x.copy_(hb, non_blocking=True)
                        else:
                            v.x.copy_(torch.from_numpy(x_in.copy()).view(v.x.shape).to(v.x.dtype), non_blocking=False)
                    solo = alone and v.solo_graph is not None
                    toks = None
                    for i in range(job.steps if gen else 1):
                        if i:   # generate: the previous run's ids are this run's input, on the device
                            v.x.copy_(o.reshape(v.x.shape))
                        outs = v.outputs
                        if solo:
                            v.solo_graph.replay()
                            outs = v.solo_outputs
                            t.solo_completed += 1
                        elif v.graph is not None:
                            v.graph.replay()
                        else:
                            v.outputs = outs = v.model(v.x)
                        if gen:
                            o = fed(outs)
                            if toks is None:
                                toks = torch.empty((job.steps,) + tuple(o.shape), dtype=o.dtype, device=o.device)
                            toks[i].copy_(o)
                    if gen:
                        fetch = [_fetch_start(toks, v.host, "gen")]
                    else:
                        fetch = [_fetch_start(outs[i], v.host, ("out", solo, i))
                                 for i in self._selected(range(len(outs)), job.want_outputs)]
                    counters = self._counters_start(t) if t.state else None
                s.synchronize()
            if job.want_outputs:
                job.outputs = [f() for f in fetch]
            if t.state:
                job.state = counters()
                for name, rows in t.pos_limits.items():
                    over = [p for p in job.state.get(name, ()) if p > rows]
                    if over:
                        raise RuntimeError(f"context full: position {max(over)} is past the {rows} cache rows "
                                           f"(state {name!r}); reset the tenant or start a new sequence")

    @staticmethod
    def _selected(items, want) -> list:
        """The outputs a request asked for: all (``True``), none, or the listed
        indices (negative ones count from the end; out-of-range ones dropped)."""
        items = list(items)
        if not want:
            return []
        if want is True:
            return items
        return [items[i] for i in want if -len(items) <= i < len(items)]

    def _counters(self, t: Tenant) -> dict:
        """A stateful tenant's small i32 states (its positions), read back
        after the run the lane has synchronised."""
        import torch

        return {k: [int(v) for v in st.cpu().tolist()] for k, st in t.state.items()
                if st.dtype == torch.int32 and st.numel() <= 64}

    def _counters_start(self, t: Tenant):
        """``_counters`` behind the lane's one synchronisation: the copies are
        queued on the current stream into pinned buffers; the returned
        function reads them once the stream is synchronised."""
        import torch

        bufs = {}
        for k, st in t.state.items():
            if st.dtype == torch.int32 and st.numel() <= 64:
                hb = bufs[k] = _pinned(t.host, ("state", k), st.shape, st.dtype)
                hb.copy_(st, non_blocking=True)
        return lambda: {k: [int(v) for v in hb.tolist()] for k, hb in bufs.items()}

    def _reset_state(self, t: Tenant) -> None:
        """Zero a tenant's state (a new sequence at position 0).  Its requests
        arrive on its one connection, one at a time, so no run of it is in
        flight; the zeroing runs on its own stream and is waited for."""
        import torch

        if not self.gpu:
            for st in t.state.values():
                st.zero_()
            return
        s = t.stream.torch if t.stream is not None else self._setup_stream
        with torch.cuda.stream(s):
            for st in t.state.values():
                st.zero_()
        s.synchronize()

    def _run_trainer(self, job: _Job, lane) -> None:
        """A training tenant's request: one optimisation step (payload =
        input + target) or a forward pass with the current weights."""
        import torch

        tr = job.tenant.trainer
        ids = str(tr.x.dtype) == "torch.int32"
        nb = job.x_bytes if job.kind == "train" else len(job.payload)
        x = None
        if nb:
            x = np.frombuffer(job.payload[:nb], dtype=np.int32 if ids else np.float32)
            if x.size != tr.x.numel():
                raise ValueError(f"input has {x.size} values, the tenant's model takes {tr.x.numel()}")
            t = job.tenant
            if ids and t.id_bound is not None and x.size and (x.min() < 0 or x.max() >= t.id_bound):
                raise ValueError(f"token ids must lie in [0, {t.id_bound})")
            x = torch.from_numpy(x.copy())
        y = None
        if job.kind == "train":
            ci = tr.spec["target_dtype"] == "i32"
            y = np.frombuffer(job.payload[nb:], dtype=np.int32 if ci else np.float32)
            if y.size != tr.y.numel():
                raise ValueError(f"target has {y.size} values, the trained output takes {tr.y.numel()}")
            if ci and y.size and (y.min() < 0 or y.max() >= tr.prog.values[tr.prog.outputs[tr.spec["output"]]].shape[-1]):
                raise ValueError("class ids must index the logits")
            y = torch.from_numpy(y.copy())
        s = job.tenant.stream.torch if (self.gpu and job.tenant.stream is not None) else lane
        ctx = torch.cuda.stream(s) if self.gpu else contextlib.nullcontext()
        with ctx:
            if job.kind == "train":
                loss = tr.step(x, y)
                if self.gpu:
                    s.synchronize()
                job.loss = float(loss.detach())
            else:
                outs = tr.forward(x)
                if self.gpu:
                    s.synchronize()
                if job.want_outputs:
                    job.outputs = [o.detach().float().cpu().numpy() for o in outs]


__all__ = ["PodServer", "Tenant", "AdmissionError", "DEFAULT_LANES", "DEFAULT_MAX_TENANTS"]
