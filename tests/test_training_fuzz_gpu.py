"""Fuzzed training tenants (hypothesis): random MLP-class programs --
linear chains with activations, LayerNorm / RMSNorm, residuals -- trained
for three steps with a random loss and optimizer on the GPU pod server
(forward + backward + step as one captured graph, gfx950 kernels for the
GEMMs) and on a CPU pod server (PyTorch fp32), the same data: the losses
agree step for step, and a YOLOS co-tenant on the GPU answers bit for bit."""
from __future__ import annotations

import math
import tempfile
from pathlib import Path

import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

pytestmark = pytest.mark.gpu

from nos_amd.podserver.client import PodClient  # noqa: E402
from nos_amd.podserver.program import Builder  # noqa: E402

WIDTH = (32, 64, 96, 160)


@st.composite
def training_cases(draw):
    seed = draw(st.integers(0, 2 ** 16))
    rng = np.random.default_rng(seed)
    B, S, D = draw(st.sampled_from((1, 2))), draw(st.sampled_from((1, 7, 33))), draw(st.sampled_from(WIDTH))
    b = Builder("fuzz-train")
    x = b.input("x", [B, S, D])
    W = lambda *shape, scale=None: b.param(f"w{len(b.params)}",   # noqa: E731
                                           rng.standard_normal(shape) * (scale or 1 / math.sqrt(shape[-1])))
    h, width = x, D
    for _ in range(draw(st.integers(1, 3))):
        kind = draw(st.sampled_from(("linear", "linear", "norm", "residual")))
        if kind == "linear":
            n = draw(st.sampled_from(WIDTH))
            act = draw(st.sampled_from((None, "relu", "gelu")))
            bias = W(n, scale=0.1) if draw(st.booleans()) else None
            h = b.op("linear", *([h, W(n, width)] + ([bias] if bias is not None else [])), act=act)
            width = n
        elif kind == "norm":
            if draw(st.booleans()):
                h = b.op("layernorm", h, W(width, scale=0.1), W(width, scale=0.1), eps=1e-5)
            else:
                h = b.op("rmsnorm", h, b.param(f"w{len(b.params)}", 1 + 0.1 * rng.standard_normal(width)), eps=1e-5)
        elif width == D:
            h = b.op("add", b.op("linear", h, W(width, width), act="relu"), h)
    classes = draw(st.sampled_from((2, 33, 64)))
    loss = draw(st.sampled_from(("mse", "cross_entropy")))
    if loss == "cross_entropy":
        h = b.op("linear", h, W(classes, width))
    prog, w = b.build([h])
    opt = draw(st.sampled_from((dict(optimizer="sgd", lr=0.05, momentum=0.9), dict(optimizer="adam", lr=1e-2),
                                dict(optimizer="adamw", lr=1e-2, weight_decay=0.01))))
    xs = [rng.standard_normal((B, S, D)).astype(np.float32) for _ in range(3)]
    if loss == "mse":
        ts = [rng.standard_normal((B, S, width)).astype(np.float32) for _ in range(3)]
    else:
        ts = [rng.integers(0, classes, (B, S)).astype(np.int32) for _ in range(3)]
    return prog, w, dict(loss=loss, **opt), xs, ts


@pytest.fixture(scope="module")
def servers():
    from nos_amd.models.yolos_program import demo_tenant
    from nos_amd.podserver.server import PodServer

    torch.backends.cuda.matmul.allow_tf32 = False
    d = Path(tempfile.mkdtemp(prefix="nos_tf_", dir="/tmp"))
    gpu = PodServer(d / "g.sock", device="cuda", lanes=4, memory_gb=64).start()
    cpu = PodServer(d / "c.sock", device="cpu", lanes=2).start()
    y = PodClient(gpu.path, connect_timeout_s=60)
    y.register("yolos", *demo_tenant("fp32", 0, small=True), memory_limit_gb=4)
    first = y.infer(outputs=True)[0]
    yield gpu, cpu, y, first
    y.close()
    gpu.stop()
    cpu.stop()


RAN: list = []


@settings(max_examples=40, deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large, HealthCheck.function_scoped_fixture])
@given(case=training_cases())
def test_fuzzed_training_tenants_match_cpu_training(servers, case):
    gpu, cpu, yolos, first = servers
    prog, w, spec, xs, ts = case
    cg = PodClient(gpu.path, connect_timeout_s=30)
    cc = PodClient(cpu.path, connect_timeout_s=30)
    try:
        cg.register("t", prog, w, memory_limit_gb=2, train=spec)
        cc.register("t", prog, w, memory_limit_gb=2, train=spec)
        for x, t in zip(xs, ts):
            lg, lc = cg.train_step(x, t)["loss"], cc.train_step(x, t)["loss"]
            np.testing.assert_allclose(lg, lc, rtol=5e-4, atol=1e-5)
    finally:
        cg.close()
        cc.close()
    RAN.append(spec["loss"])
    assert all(np.array_equal(a, b_) for a, b_ in zip(yolos.infer(outputs=True)[0], first))


def test_training_fuzz_covered_both_losses(servers):
    assert len(RAN) >= 30 and {"mse", "cross_entropy"} <= set(RAN), RAN
