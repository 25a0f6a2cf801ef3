"""Training tenants on the GPU pod server: forward + backward + optimizer
step captured into one HIP graph per tenant, replayed on the lanes beside
inference tenants; losses follow torch.optim on the same GPU."""
from __future__ import annotations

import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from nos_amd.models.llama_program import llama_config, llama_model, llama_program  # noqa: E402
from nos_amd.models.yolos_program import demo_tenant  # noqa: E402
from nos_amd.podserver.client import PodClient  # noqa: E402
from nos_amd.podserver.export import export  # noqa: E402
from nos_amd.podserver.server import PodServer  # noqa: E402

from test_training_tenants import Mlp, _data  # noqa: E402


@pytest.fixture(autouse=True)
def _no_tf32():
    torch.backends.cuda.matmul.allow_tf32 = False
    yield


@pytest.mark.parametrize("opt", [dict(optimizer="sgd", lr=0.05, momentum=0.9),
                                 dict(optimizer="sgd", lr=0.05, momentum=0.9, nesterov=True),
                                 dict(optimizer="adam", lr=1e-2, weight_decay=0.01),
                                 dict(optimizer="adamw", lr=1e-2, weight_decay=0.01)])
def test_graphed_training_tenant_beside_an_inference_tenant(tmp_path, opt):
    torch.manual_seed(0)
    m = Mlp()
    prog, w = export(copy.deepcopy(m), torch.zeros(4, 8, 32), name="mlp")
    srv = PodServer(tmp_path / "s.sock", device="cuda", lanes=4, memory_gb=64).start()
    try:
        c = PodClient(srv.path, connect_timeout_s=30)
        rep = c.register("trainer", prog, w, memory_limit_gb=1, train=dict(loss="mse", **opt))
        assert rep["compile"]["graph"] is True
        y = PodClient(srv.path, connect_timeout_s=30)
        y.register("yolos", *demo_tenant("fp32", 0, small=False), memory_limit_gb=2)
        ref = copy.deepcopy(m).cuda().train()
        if opt["optimizer"] == "sgd":
            ro = torch.optim.SGD(ref.parameters(), lr=opt["lr"], momentum=opt["momentum"],
                                 nesterov=opt.get("nesterov", False))
        else:
            cls = torch.optim.AdamW if opt["optimizer"] == "adamw" else torch.optim.Adam
            ro = cls(ref.parameters(), lr=opt["lr"], weight_decay=opt["weight_decay"])
        for k, (x, t) in enumerate(_data(1, 6)):
            r = c.train_step(x, t)
            y.infer()
            ro.zero_grad()
            loss = torch.nn.functional.mse_loss(ref(torch.from_numpy(x).cuda()), torch.from_numpy(t).cuda())
            loss.backward()
            ro.step()
            assert r["step"] == k + 1
            np.testing.assert_allclose(r["loss"], float(loss.detach()), rtol=1e-4)
        x = _data(9, 1)[0][0]
        out, _ = c.infer(x, outputs=True)
        with torch.no_grad():
            np.testing.assert_allclose(out[0], ref(torch.from_numpy(x).cuda()).cpu().numpy(), rtol=1e-3, atol=1e-4)
        c.close()
        y.close()
    finally:
        srv.stop()


def test_graphed_decoder_fine_tuning(tmp_path):
    torch.manual_seed(0)
    m = llama_model(llama_config(False), 0)
    prog, w = llama_program(m, 16)
    srv = PodServer(tmp_path / "s.sock", device="cuda", lanes=2, memory_gb=64).start()
    try:
        c = PodClient(srv.path, connect_timeout_s=30)
        c.register("lm", prog, w, memory_limit_gb=2, train={"loss": "cross_entropy", "optimizer": "adamw", "lr": 3e-3})
        ref = copy.deepcopy(m).cuda().train()
        ro = torch.optim.AdamW(ref.parameters(), lr=3e-3)
        g = np.random.default_rng(3)
        V = m.config.vocab_size
        first = None
        ids = g.integers(0, V, (1, 17)).astype(np.int32)
        for _ in range(8):   # one batch, over and over: the loss must fall
            r = c.train_step(ids[:, :16], ids[:, 1:])
            ro.zero_grad()
            logits = ref(torch.from_numpy(ids[:, :16]).long().cuda()).logits
            loss = torch.nn.functional.cross_entropy(logits.reshape(-1, V),
                                                     torch.from_numpy(ids[:, 1:]).long().cuda().reshape(-1))
            loss.backward()
            ro.step()
            np.testing.assert_allclose(r["loss"], float(loss.detach()), rtol=1e-3)
            first = first or r["loss"]
        assert r["loss"] < 0.9 * first
        c.close()
    finally:
        srv.stop()


def test_trainer_captures_while_other_tenants_replay_and_on_a_cu_slice(tmp_path):
    """A training tenant registers (warm-up + graph capture) while an
    inference tenant replays continuously on the lanes, on its own CU-masked
    stream; both keep answering correctly."""
    import threading

    torch.manual_seed(1)
    m = Mlp()
    prog, w = export(copy.deepcopy(m), torch.zeros(4, 8, 32), name="mlp")
    srv = PodServer(tmp_path / "s.sock", device="cuda", lanes=4, memory_gb=64).start()
    stop = threading.Event()
    errors = []
    try:
        y = PodClient(srv.path, connect_timeout_s=30)
        y.register("yolos", *demo_tenant("fp32", 0, small=False), memory_limit_gb=2)
        y.infer()

        def spin():
            try:
                while not stop.is_set():
                    y.infer()
            except Exception as e:  # noqa: BLE001 -- reported below
                errors.append(e)

        th = threading.Thread(target=spin, daemon=True)
        th.start()
        c = PodClient(srv.path, connect_timeout_s=30)
        rep = c.register("trainer", prog, w, memory_limit_gb=1, cu_mask="0xffffffff",
                         train={"loss": "mse", "optimizer": "sgd", "lr": 0.05, "momentum": 0.9})
        assert rep["compile"]["graph"] is True and rep["cu_mask"] == "0xffffffff"
        ref = copy.deepcopy(m).cuda().train()
        ro = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9)
        for x, t in _data(2, 4):
            r = c.train_step(x, t)
            ro.zero_grad()
            loss = torch.nn.functional.mse_loss(ref(torch.from_numpy(x).cuda()), torch.from_numpy(t).cuda())
            loss.backward()
            ro.step()
            np.testing.assert_allclose(r["loss"], float(loss.detach()), rtol=1e-4)
        stop.set()
        th.join(timeout=60)
        assert not errors, errors
        c.close()
        y.close()
    finally:
        stop.set()
        srv.stop()


def test_graphed_checkpoint_resume_continues_the_run(tmp_path):
    """GPU: a resumed training tenant's captured graph starts from the
    checkpoint's weights and AdamW moments (the capture's warm-up restores
    them in place), so 3 + 3 steps equal 6 uninterrupted ones."""
    torch.manual_seed(4)
    prog, w = export(Mlp(), torch.zeros(4, 8, 32), name="mlp")
    data = _data(6, 6)
    spec = {"loss": "mse", "optimizer": "adamw", "lr": 1e-2}
    srv = PodServer(tmp_path / "s.sock", device="cuda", lanes=2, memory_gb=64).start()
    try:
        a = PodClient(srv.path, connect_timeout_s=30)
        a.register("a", prog, w, memory_limit_gb=1, train=spec)
        straight = [a.train_step(x, y)["loss"] for x, y in data]
        a.close()
        b = PodClient(srv.path, connect_timeout_s=30)
        b.register("b", prog, w, memory_limit_gb=1, train=spec)
        first = [b.train_step(x, y)["loss"] for x, y in data[:3]]
        ck = b.checkpoint()
        b.close()
        c = PodClient(srv.path, connect_timeout_s=30)
        c.register("c", prog, ck, memory_limit_gb=1, train={**spec, "resume": True})
        rest = [c.train_step(x, y)["loss"] for x, y in data[3:]]
        np.testing.assert_allclose(first + rest, straight, rtol=1e-5)
        c.close()
    finally:
        srv.stop()
