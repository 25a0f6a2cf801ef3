"""Training tenants on the pod server (podserver/training.py): a program plus
a training spec; the server runs whole optimisation steps in the shared
context and matches the same model trained by plain torch.optim."""
from __future__ import annotations

import copy

import numpy as np
import pytest
import torch
import torch.nn as nn

from nos_amd.models.llama_program import llama_config, llama_model, llama_program
from nos_amd.podserver import program as PG
from nos_amd.podserver.client import PodClient, PodServerError
from nos_amd.podserver.export import export
from nos_amd.podserver.server import PodServer
from nos_amd.podserver.training import parse_train_spec, train_bytes_estimate


class Mlp(nn.Module):
    def __init__(self):
        super().__init__()
        self.ln = nn.LayerNorm(32)
        self.fc1 = nn.Linear(32, 64)
        self.fc2 = nn.Linear(64, 16)

    def forward(self, x):
        return self.fc2(torch.nn.functional.gelu(self.fc1(self.ln(x))))


@pytest.fixture
def server(tmp_path):
    srv = PodServer(tmp_path / "s.sock", device="cpu", lanes=2, memory_gb=40).start()
    yield srv
    srv.stop()


def _data(seed, n=5):
    g = np.random.default_rng(seed)
    return [(g.standard_normal((4, 8, 32)).astype(np.float32), g.standard_normal((4, 8, 16)).astype(np.float32))
            for _ in range(n)]


@pytest.mark.parametrize("opt", [dict(optimizer="sgd", lr=0.05, momentum=0.9),
                                 dict(optimizer="sgd", lr=0.05, momentum=0.9, nesterov=True),
                                 dict(optimizer="adam", lr=1e-2, weight_decay=0.01),
                                 dict(optimizer="adamw", lr=1e-2, weight_decay=0.01)])
def test_training_tenant_matches_torch_optim(server, opt):
    torch.manual_seed(0)
    m = Mlp()
    prog, w = export(copy.deepcopy(m), torch.zeros(4, 8, 32), name="mlp")
    c = PodClient(server.path, connect_timeout_s=5)
    rep = c.register("trainer", prog, w, memory_limit_gb=1, train=dict(loss="mse", **opt))
    assert rep["compile"]["train"] == opt["optimizer"]
    ref = copy.deepcopy(m).train()
    if opt["optimizer"] == "sgd":
        ro = torch.optim.SGD(ref.parameters(), lr=opt["lr"], momentum=opt["momentum"],
                             nesterov=opt.get("nesterov", False))
    else:
        cls = torch.optim.AdamW if opt["optimizer"] == "adamw" else torch.optim.Adam
        ro = cls(ref.parameters(), lr=opt["lr"], weight_decay=opt["weight_decay"])
    for k, (x, y) in enumerate(_data(1)):
        r = c.train_step(x, y)
        ro.zero_grad()
        loss = torch.nn.functional.mse_loss(ref(torch.from_numpy(x)), torch.from_numpy(y))
        loss.backward()
        ro.step()
        assert r["step"] == k + 1
        np.testing.assert_allclose(r["loss"], float(loss.detach()), rtol=1e-5)
    x = _data(9, 1)[0][0]
    out, _ = c.infer(x, outputs=True)
    with torch.no_grad():
        np.testing.assert_allclose(out[0], ref(torch.from_numpy(x)).numpy(), rtol=1e-4, atol=1e-5)
    # the weights resume: an inference tenant on them answers like the trained model
    wb = c.weights()
    assert len(wb) == len(w) and wb != w
    c2 = PodClient(server.path, connect_timeout_s=5)
    c2.register("served", prog, wb, memory_limit_gb=1)
    out2, _ = c2.infer(x, outputs=True)
    np.testing.assert_allclose(out2[0], out[0], rtol=1e-4, atol=1e-5)
    st = c.stats()
    kinds = {t["pod"]: (t["kind"], t["train_steps"]) for t in st["tenants"]}
    assert kinds == {"trainer": ("train", 5), "served": ("infer", 0)}
    with pytest.raises(PodServerError, match="needs a training tenant"):
        c2.train_step(x, _data(1, 1)[0][1])
    c.close()
    c2.close()


def test_decoder_fine_tunes_with_cross_entropy(server):
    """A Llama program as a causal-LM training tenant: next-token cross
    entropy over token-id inputs, AdamW; rotary tables stay frozen; losses
    follow the transformers model trained the same way."""
    torch.manual_seed(0)
    m = llama_model(llama_config(False), 0)
    prog, w = llama_program(m, 16)
    spec = parse_train_spec({"loss": "cross_entropy", "optimizer": "adamw", "lr": 3e-3}, PG.parse(prog, w))
    assert {"rope.cos", "rope.sin"} <= set(spec["frozen"]) and spec["target_shape"] == (1, 16)
    c = PodClient(server.path, connect_timeout_s=5)
    c.register("lm", prog, w, memory_limit_gb=2, train={"loss": "cross_entropy", "optimizer": "adamw", "lr": 3e-3})
    ref = copy.deepcopy(m).train()
    ro = torch.optim.AdamW(ref.parameters(), lr=3e-3)
    g = np.random.default_rng(3)
    V = m.config.vocab_size
    losses = []
    for _ in range(4):
        ids = g.integers(0, V, (1, 17)).astype(np.int32)
        r = c.train_step(ids[:, :16], ids[:, 1:])
        ro.zero_grad()
        logits = ref(torch.from_numpy(ids[:, :16]).long()).logits
        loss = torch.nn.functional.cross_entropy(logits.reshape(-1, V), torch.from_numpy(ids[:, 1:]).long().reshape(-1))
        loss.backward()
        ro.step()
        np.testing.assert_allclose(r["loss"], float(loss.detach()), rtol=2e-4)
        losses.append(r["loss"])
    with pytest.raises(PodServerError, match="class ids must index the logits"):
        c.train_step(ids[:, :16], np.full((1, 16), V, np.int32))
    c.close()


def test_train_specs_are_validated_before_allocation(server):
    prog, w = export(Mlp(), torch.zeros(4, 8, 32), name="mlp")
    p = PG.parse(prog, w)
    for bad, match in (({"loss": "hinge"}, "train.loss"), ({"lr": 0}, "train.lr"), ({"lr": float("nan")}, "train.lr"),
                       ({"frozen": ["nope"]}, "train.frozen"), ({"schedule": 1}, "unknown train keys"),
                       ({"loss": "cross_entropy", "output": 3}, "train.output"),
                       ({"nesterov": True}, "train.nesterov"), ({"resume": "false"}, "train.resume"),
                       ({"optimizer": "sgd", "momentum": 0.9, "nesterov": "false"}, "train.nesterov")):
        with pytest.raises(PG.ProgramError, match=match):
            parse_train_spec(bad, p)
    spec = parse_train_spec({"optimizer": "adamw"}, p)
    est = train_bytes_estimate(p, spec)
    assert est > 4 * p.param_bytes   # weights + grads + two Adam states + activations
    c = PodClient(server.path, connect_timeout_s=5)
    with pytest.raises(PodServerError, match="static estimate"):
        c.register("big", prog, w, memory_limit_gb=est / 2 ** 30 / 2, train={"optimizer": "adamw"})
    with pytest.raises(PodServerError, match="no variants"):
        c.register("v", prog, w, memory_limit_gb=1, train={}, variants=[prog])
    c.close()


def test_bf16_program_trains_in_fp32_and_checkpoints_in_its_wire_dtype(server):
    torch.manual_seed(2)
    prog, w = export(Mlp(), torch.zeros(4, 8, 32), name="mlp16", dtype="bf16")
    c = PodClient(server.path, connect_timeout_s=5)
    c.register("t16", prog, w, memory_limit_gb=1, train={"optimizer": "adamw", "lr": 1e-2})
    losses = [c.train_step(x, y)["loss"] for x, y in _data(4, 1) * 6]   # one batch, six times
    assert losses[-1] < losses[0]
    wb = c.weights()
    assert len(wb) == len(w) and wb != w
    c2 = PodClient(server.path, connect_timeout_s=5)
    c2.register("s16", prog, wb, memory_limit_gb=1)
    out, _ = c2.infer(_data(4, 1)[0][0], outputs=True)
    assert np.isfinite(out[0]).all()
    c.close()
    c2.close()


@pytest.mark.parametrize("opt", [dict(optimizer="sgd", lr=0.05, momentum=0.9), dict(optimizer="adamw", lr=1e-2)])
def test_checkpoint_resumes_weights_and_optimizer_state(server, opt):
    """Train 3 steps, checkpoint, resume in a new tenant for 3 more: the
    losses equal 6 uninterrupted steps (momentum / Adam moments carried)."""
    torch.manual_seed(3)
    prog, w = export(Mlp(), torch.zeros(4, 8, 32), name="mlp")
    data = _data(5, 6)
    spec = dict(loss="mse", **opt)
    a = PodClient(server.path, connect_timeout_s=5)
    a.register("a", prog, w, memory_limit_gb=1, train=spec)
    straight = [a.train_step(x, y)["loss"] for x, y in data]
    a.close()
    b = PodClient(server.path, connect_timeout_s=5)
    b.register("b", prog, w, memory_limit_gb=1, train=spec)
    first = [b.train_step(x, y)["loss"] for x, y in data[:3]]
    ck = b.checkpoint()
    b.close()
    c = PodClient(server.path, connect_timeout_s=5)
    c.register("c", prog, ck, memory_limit_gb=1, train={**spec, "resume": True})
    rest = [c.train_step(x, y)["loss"] for x, y in data[3:]]
    np.testing.assert_allclose(first + rest, straight, rtol=1e-6)
    c.close()
    d = PodClient(server.path, connect_timeout_s=5)
    with pytest.raises(PodServerError, match="resume payload"):
        d.register("d", prog, w, memory_limit_gb=1, train={**spec, "resume": True})
    d.close()


def test_adam_step_count_checkpoints_exactly_past_float32_range(server):
    """Adam's step is stored as two exact float32 slots, so
    a count above 2^24 survives checkpoint -> resume."""
    from nos_amd.podserver.training import Trainer

    prog, w = export(Mlp(), torch.zeros(4, 8, 32), name="mlp")
    p = PG.parse(prog, w)
    spec = parse_train_spec({"optimizer": "adamw"}, p)
    tr = Trainer(p, spec, "cpu")
    x, y = _data(4, 1)[0]
    tr.step(torch.from_numpy(x), torch.from_numpy(y))
    big = (1 << 24) + 3
    for st in tr.opt.state.values():   # float32 cannot hold 2^24 + 3: an exact count to checkpoint
        st["step"] = torch.tensor(float(big), dtype=torch.float64)
    ck = tr.checkpoint_bytes()
    tr2 = Trainer(p, {**spec, "resume": True}, "cpu", ck[len(w):])
    steps = {float(st["step"]) for st in tr2.opt.state.values()}
    assert steps == {float(np.float32(big))}   # restored into torch's float32 step tensor from the exact count
    raw = np.frombuffer(ck[len(w):], np.float32)
    assert (1.0 in raw) and (3.0 in raw)         # hi = 1, lo = 3: the exact split
