"""Stateful decoder tenants on the pod server (CPU): K / V caches and a
position counter that persist across requests (program ``state``; ops
``kv_write`` / ``rotary_at`` / ``sdpa_cache`` / ``pos_add`` / ``pos_set`` /
``argmax``), a prefill program and a one-token decode program over the same
weights and state, and greedy generation that matches
``transformers.LlamaForCausalLM.generate`` token for token.

Reference: an MPS client is any CUDA process
(``/root/reference/docs/en/docs/dynamic-gpu-partitioning/partitioning-modes-comparison.md:29-34``);
LLM serving -- token-by-token generation over a KV cache -- is the dominant
fractional-GPU workload such a client runs.
"""
from __future__ import annotations

import copy

import numpy as np
import pytest
import torch

from nos_amd.models.llama_program import llama_config, llama_decode_programs, llama_model
from nos_amd.podserver import program as PG
from nos_amd.podserver.client import PodClient, PodServerError
from nos_amd.podserver.server import PodServer

MAX_LEN = 64


@pytest.fixture(scope="module")
def model():
    return llama_model(llama_config(False), 0)


@pytest.fixture(scope="module")
def tenant(model):
    return llama_decode_programs(model, 8, MAX_LEN, extend=(4,))


@pytest.fixture
def server(tmp_path):
    srv = PodServer(tmp_path / "s.sock", device="cpu", lanes=2, memory_gb=40).start()
    yield srv
    srv.stop()


def _hf_generate(model, prompt: np.ndarray, n: int) -> np.ndarray:
    ids = torch.from_numpy(prompt.astype(np.int64))
    out = model.generate(ids, max_new_tokens=n, do_sample=False, pad_token_id=0, min_new_tokens=n)
    return out[:, prompt.shape[1]:].numpy()


def _prompt(seed: int, b: int = 1, n: int = 8) -> np.ndarray:
    return np.random.default_rng(seed).integers(0, 512, (b, n)).astype(np.int32)


def test_server_generation_matches_hf_generate_token_for_token(model, tenant, server):
    """The verdict's bar: greedy generation of 32 tokens from an 8-token
    prompt on the pod server equals LlamaForCausalLM.generate."""
    progs, w = tenant
    c = PodClient(server.path, connect_timeout_s=5)
    rep = c.register("llm", progs[0], w, memory_limit_gb=1, variants=progs[1:])
    assert sorted(map(tuple, rep["input_shapes"])) == [(1, 1), (1, 4), (1, 8)]
    prompt = _prompt(0)
    ids, tm = c.generate(prompt, 32)
    assert np.array_equal(ids, _hf_generate(model, prompt, 32))
    assert tm["state"] == {"pos": [8 + 31]}
    assert len(tm["step_s"]) == 31
    c.close()


def test_server_loop_equals_per_token_requests(model, tenant, server):
    """generate(server_loop=True): ONE request runs the decode steps in the
    server, ids fed back on the device -- the same tokens and final position
    as a request per token; bad generate requests are refused."""
    progs, w = tenant
    c = PodClient(server.path, connect_timeout_s=5)
    c.register("llm", progs[0], w, memory_limit_gb=1, variants=progs[1:])
    p = _prompt(7)
    a, ta = c.generate(p, 20, server_loop=True)
    b, tb = c.generate(p, 20, server_loop=False)
    assert np.array_equal(a, b) and ta["state"] == tb["state"] == {"pos": [8 + 19]}
    for bad in ({"steps": 0}, {"steps": 5000}, {"steps": True}, {"steps": 2, "output": 9}):
        with pytest.raises(PodServerError):
            c._call({"op": "generate", "shape": [1, 1], "dtype": "i32", "output": 1, **bad},
                    np.array([[1]], np.int32).tobytes())
    c.close()
    m = PodClient(server.path, connect_timeout_s=5)     # a stateless tenant has no decode loop
    from nos_amd.podserver.program import mlp_program

    prog, wb = mlp_program(dim=16, layers=1, batch=4, dtype="fp32")
    m.register("mlp", prog, wb, memory_limit_gb=1)
    with pytest.raises(PodServerError, match="stateful"):
        m._call({"op": "generate", "steps": 2}, b"")
    m.close()


def test_reset_starts_a_new_sequence_and_repeats_it(model, tenant, server):
    progs, w = tenant
    c = PodClient(server.path, connect_timeout_s=5)
    c.register("llm", progs[0], w, memory_limit_gb=1, variants=progs[1:])
    p = _prompt(1)
    a, _ = c.generate(p, 12)
    assert c.reset()["state"] == {"pos": [0]}
    b, _ = c.generate(p, 12)            # prefill resets too; the explicit reset zeroed the caches as well
    assert np.array_equal(a, b)
    c.close()


def test_a_longer_prompt_runs_as_prefill_plus_extend_chunks(model, tenant, server):
    """A 12-token prompt = the 8-token prefill + one 4-token extend step at
    the device-side position 8 (sdpa_cache over cached + new keys)."""
    progs, w = tenant
    c = PodClient(server.path, connect_timeout_s=5)
    c.register("llm", progs[0], w, memory_limit_gb=1, variants=progs[1:])
    p = _prompt(2, n=12)
    c.infer(p[:, :8], outputs=[1])
    outs, rep = c.infer(p[:, 8:], outputs=[1])
    assert rep["state"] == {"pos": [12]}
    first = int(outs[0].reshape(-1)[0])
    ids = [first]
    for _ in range(9):
        o, _ = c.infer(np.array([[ids[-1]]], np.int32), outputs=[1])
        ids.append(int(o[0].reshape(-1)[0]))
    assert ids == _hf_generate(model, p, 10)[0].tolist()
    c.close()


def test_interleaved_tenants_keep_their_own_state(model, tenant, server):
    progs, w = tenant
    cs = [PodClient(server.path, connect_timeout_s=5) for _ in range(2)]
    for i, c in enumerate(cs):
        c.register(f"llm{i}", progs[0], w, memory_limit_gb=1, variants=progs[1:])
    ps = [_prompt(10), _prompt(11)]
    toks = [[int(c.infer(p, outputs=[1])[0][0].reshape(-1)[0])] for c, p in zip(cs, ps)]
    for _ in range(15):
        for c, t in zip(cs, toks):
            t.append(int(c.infer(np.array([[t[-1]]], np.int32), outputs=[1])[0][0].reshape(-1)[0]))
    for p, t in zip(ps, toks):
        assert t == _hf_generate(model, p, 16)[0].tolist()
    for c in cs:
        c.close()


def test_batch_two_sequences(model):
    """B = 2: one position per sequence, both advanced by each step."""
    progs, w = llama_decode_programs(model, 6, MAX_LEN, batch=2)
    ps = PG.parse_variants(progs, w)
    params = ps[0].tensors("cpu")
    state = ps[0].state_tensors("cpu")
    pre, step = (p.compile("cpu", params=params, state=state) for p in ps)
    prompt = _prompt(3, b=2, n=6)
    tok = pre(torch.from_numpy(prompt))[1].reshape(2, 1)
    out = [tok]
    for _ in range(7):
        tok = step(tok.to(torch.int32))[1].reshape(2, 1)
        out.append(tok)
    assert state["pos"].tolist() == [13, 13]
    assert np.array_equal(torch.cat(out, 1).numpy(), _hf_generate(model, prompt, 8))


def test_generation_past_the_cache_is_reported_not_corrupting(model, server):
    progs, w = llama_decode_programs(model, 8, 16)
    c = PodClient(server.path, connect_timeout_s=5)
    c.register("llm", progs[0], w, memory_limit_gb=1, variants=progs[1:])
    ids, tm = c.generate(_prompt(4), 8)            # positions 8 .. 15: the cache's last row
    assert tm["state"] == {"pos": [15]}
    c.infer(ids[:, -1:], outputs=[1])              # writes row 15, position 16 = full, still exact
    with pytest.raises(PodServerError, match="context full"):
        c.infer(ids[:, -1:], outputs=[1])          # row 16 does not exist: refused
    c.reset()
    again, _ = c.generate(_prompt(4), 8)
    assert np.array_equal(again, ids)
    c.close()


def test_the_state_counts_against_the_slice(model):
    progs, w = llama_decode_programs(model, 8, 4096)
    ps = PG.parse_variants(progs, w)
    # 2 layers x K, V x [1, 4096, 1, 128] fp32 = 8 MiB of cache
    assert ps[0].state_bytes == 2 * 2 * 4096 * 128 * 4 + 4
    assert all(p.bytes_estimate > p.state_bytes + p.param_bytes for p in ps)
    small = llama_decode_programs(model, 8, 64)[0]
    assert PG.parse(small[0], w).bytes_estimate < ps[0].bytes_estimate


def test_a_cache_larger_than_the_slice_is_refused_at_registration(model, server):
    progs, w = llama_decode_programs(model, 8, 1 << 17)    # 2 x 2 x 128k x 128 x 4 B = 256 MiB
    c = PodClient(server.path, connect_timeout_s=5)
    with pytest.raises(PodServerError, match="static estimate"):
        c.register("big", progs[0], w, memory_limit_gb=0.2, variants=progs[1:])
    c.close()


def _bad(prog: dict, mutate) -> dict:
    p = copy.deepcopy(prog)
    mutate(p)
    return p


@pytest.mark.parametrize("mutate, match", [
    # a later node reads the cache version a kv_write already replaced
    (lambda p: p["nodes"].insert(len(p["nodes"]) - 1, {"op": "argmax", "inputs": ["kc0"], "output": "z"}),
     "updated in place"),
    (lambda p: p["outputs"].append("pos"), "cannot be an output"),
    (lambda p: p["state"].append({"name": "x", "shape": [1], "dtype": "int8"}), "state dtype"),
    (lambda p: p["nodes"].append({"op": "pos_add", "inputs": ["logits"], "output": "q2", "attrs": {"n": 1}}),
     "i32 \\[B\\] position state"),
    (lambda p: p["nodes"].extend([{"op": "reshape", "inputs": ["next_ids"], "output": "nx", "attrs": {"shape": [1]}},
                                  {"op": "pos_add", "inputs": ["nx"], "output": "q2", "attrs": {"n": 1}}]),
     "not one"),
    (lambda p: p["nodes"].append({"op": "pos_set", "inputs": ["pos"], "output": "q2", "attrs": {"value": -1}}),
     "updated in place|value must be"),
])
def test_malformed_state_programs_are_refused(tenant, mutate, match):
    progs, w = tenant
    with pytest.raises(PG.ProgramError, match=match):
        PG.parse(_bad(progs[1], mutate), w)


def test_variants_must_share_one_state(tenant):
    progs, w = tenant
    other = _bad(progs[1], lambda p: p["state"][1].update(shape=[1, 32, 1, 128]))
    with pytest.raises(PG.ProgramError):
        PG.parse_variants([progs[0], other], w)


def test_a_stateful_program_cannot_train(tenant, server):
    progs, w = tenant
    c = PodClient(server.path, connect_timeout_s=5)
    with pytest.raises(PodServerError, match="cannot be a training tenant"):
        c.register("t", progs[1], w, memory_limit_gb=1, train={"loss": "cross_entropy"})
    c.close()


def test_static_position_zero_prefill_uses_the_flash_path(tenant):
    """The prefill's position is 0 by construction: its attention compiles to
    causal sdpa on the fresh keys (no cache reads), the decode step keeps the
    cache kernels with the rotary fused into them."""
    progs, w = tenant
    ps = PG.parse_variants(progs, w)
    params = ps[0].tensors("cpu")
    pre, step = (p.compile("cpu", params=params) for p in ps[:2])
    kinds_pre = [s.kind for s in pre.steps]
    kinds_step = [s.kind for s in step.steps]
    assert "sdpa" in kinds_pre and "sdpa_cache" not in kinds_pre and "rotary_at" not in kinds_pre
    assert kinds_pre.count("kv_write") == 4
    assert "sdpa_cache" in kinds_step and "rotary_at" not in kinds_step   # fused into kv_write / sdpa_cache
    assert step.stats["rotary_at_fused"] == 4


def test_reference_equals_hf_forward_logits(model, tenant):
    """Program.reference with an explicit state: prefill logits = HF's last-token logits."""
    progs, w = tenant
    p0 = PG.parse(progs[0], w)
    prompt = _prompt(5)
    state = {k: (t if t.dtype == torch.int32 else t.float()) for k, t in p0.state_tensors("cpu").items()}
    logits, nxt = p0.reference(torch.from_numpy(prompt), state=state)
    with torch.no_grad():
        hf = model(torch.from_numpy(prompt.astype(np.int64))).logits[:, -1:]
    torch.testing.assert_close(logits, hf, rtol=1e-4, atol=1e-4)
    assert int(state["pos"][0]) == 8 and int(nxt.reshape(-1)[0]) == int(hf.argmax(-1).reshape(-1)[0])


def test_variants_share_their_folded_and_merged_weights(tenant):
    """shape variants over one weight payload make ONE copy of
    each derived constant (RMSNorm-folded, Q / K / V and gate / up merged
    weights), not one per variant."""
    progs, w = tenant
    ps = PG.parse_variants(progs, w)
    params, state, derived = ps[0].tensors("cpu"), ps[0].state_tensors("cpu"), {}
    cps = [p.compile("cpu", params=params, state=state, derived=derived) for p in ps]

    def derived_ids(c):
        return {id(v) for k, v in c.consts.items() if "::" in k and ("merged" in k or "rms" in k)}

    a, b, e = (derived_ids(c) for c in cps)
    assert a and b == e and b <= a     # the decode / extend variants reuse the prefill's tensors


def test_stateful_tenants_are_latency_tenants_on_the_priority_lanes(tenant, server):
    """A decoder's generation steps go to the priority lanes' own queue
    (high-priority streams on a GPU); a tenant may opt out or in."""
    from nos_amd.models.yolos_program import demo_tenant

    progs, w = tenant
    a, b, y = (PodClient(server.path, connect_timeout_s=5) for _ in range(3))
    a.register("dec", progs[0], w, memory_limit_gb=1, variants=progs[1:])
    b.register("dec-bulk", progs[0], w, memory_limit_gb=1, variants=progs[1:], priority="throughput")
    y.register("yolos", *demo_tenant("fp32", 0, small=False), memory_limit_gb=1)
    kinds = {t["pod"]: t["latency"] for t in a.stats()["tenants"]}
    assert kinds == {"dec": True, "dec-bulk": False, "yolos": False}
    ids, _ = a.generate(_prompt(6), 4)
    assert ids.shape == (1, 4)
    c = PodClient(server.path, connect_timeout_s=5)
    with pytest.raises(PodServerError, match="priority must be"):
        c.register("bad", progs[0], w, memory_limit_gb=1, priority="urgent")
    for x in (a, b, y, c):
        x.close()


def test_job_queue_serves_latency_requests_first():
    """Every lane takes a waiting latency request before a throughput one; a
    priority lane takes latency requests only; close() drains, then stops."""
    import threading

    from nos_amd.podserver.server import _JobQueue

    q = _JobQueue()
    q.put("t1")
    q.put("t2")
    q.put("d1", hi=True)
    assert q.get() == "d1" and q.get() == "t1"
    got = []
    th = threading.Thread(target=lambda: got.append(q.get(hi_only=True)))
    th.start()
    th.join(0.2)
    assert th.is_alive() and not got          # t2 is not a priority lane's
    q.put("d2", hi=True)
    th.join(5)
    assert got == ["d2"] and q.qsize() == 1
    q.close()
    assert q.get() == "t2" and q.get() is None and q.get(hi_only=True) is None
    # a throughput lane beside CU-reserved priority lanes leaves latency requests to them
    q = _JobQueue()
    q.put("d1", hi=True)
    q.put("t1")
    assert q.get(lo_only=True) == "t1" and q.qsize() == 1
    q.close()
    assert q.get(lo_only=True) is None and q.get(hi_only=True) == "d1"


def test_latency_cus_must_be_xcd_symmetric(tmp_path):
    from nos_amd.podserver.server import PodServer

    for bad, pl in ((12, 2), (-8, 2), (16, 0)):
        with pytest.raises(ValueError, match="latency_cus"):
            PodServer(tmp_path / "s.sock", device="cpu", priority_lanes=pl, latency_cus=bad)
    with pytest.raises(ValueError, match="masked_queues"):
        PodServer(tmp_path / "s.sock", device="cpu", priority_lanes=2, latency_cus=16, masked_queues=0)


def test_selected_outputs():
    from nos_amd.podserver.server import PodServer

    sel = PodServer._selected
    assert sel([1, 2, 3], True) == [1, 2, 3] and sel([1, 2, 3], False) == [] and sel([1, 2, 3], None) == []
    assert sel([1, 2, 3], [0, -1, 5, -4]) == [1, 3]
