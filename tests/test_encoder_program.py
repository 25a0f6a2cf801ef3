"""A third tenant architecture through the pod server: a stack of standard
``torch.nn.TransformerEncoderLayer`` (pre-LN, GELU, batch-first) shipped as a
program (models/encoder_program.py) -- the tenant's own PyTorch module is
the reference.  CPU here; the GPU run is in tests/test_podserver_gpu.py."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from nos_amd.models.encoder_program import encoder_program, random_encoder_weights
from nos_amd.podserver import program as PG


def _torch_encoder(layers, hidden, heads, mlp, weights):
    layer = torch.nn.TransformerEncoderLayer(hidden, heads, mlp, dropout=0.0, activation="gelu", batch_first=True,
                                             norm_first=True)
    enc = torch.nn.TransformerEncoder(layer, layers, norm=torch.nn.LayerNorm(hidden), enable_nested_tensor=False)
    enc.load_state_dict({k: torch.from_numpy(v) for k, v in weights.items()})
    return enc.eval()


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_encoder_program_matches_torch_transformer_encoder(dtype):
    L, hid, heads, mlp, S = 2, 128, 2, 512, 40
    w = random_encoder_weights(L, hid, mlp, seed=1)
    prog = PG.parse(*encoder_program(w, L, heads, (2, S, hid), dtype))
    m = prog.compile("cpu")
    assert m.stats["layernorm_folded"] == 2 * L and m.stats["qkv_attention_fused"] == L
    assert m.stats["plane_handoffs"] == 2 * L  # attention -> out_proj, linear1 -> linear2 (used under h3)
    assert m.stats["residual_fused"] == 2 * L and m.stats["activation_fused"] == L
    x = torch.randn(2, S, hid, generator=torch.Generator().manual_seed(2))
    with torch.no_grad():
        ref = _torch_encoder(L, hid, heads, mlp, w)(x)
        out = m(x)[0]
    err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
    assert err < (1e-5 if dtype == "fp32" else 3e-2), err


def test_encoder_tenant_through_the_cpu_pod_server(tmp_path):
    from nos_amd.podserver.client import PodClient
    from nos_amd.podserver.server import PodServer

    L, hid, heads, mlp, S = 1, 128, 2, 256, 16
    w = random_encoder_weights(L, hid, mlp, seed=3)
    srv = PodServer(tmp_path / "s.sock", device="cpu", lanes=1, memory_gb=10).start()
    try:
        c = PodClient(srv.path, connect_timeout_s=5)
        rep = c.register("enc", *encoder_program(w, L, heads, (1, S, hid)), memory_limit_gb=1)
        x = np.random.default_rng(4).standard_normal(rep["input_shape"]).astype(np.float32)
        out, _ = c.infer(x, outputs=True)
        with torch.no_grad():
            ref = _torch_encoder(L, hid, heads, mlp, w)(torch.from_numpy(x)).numpy()
        np.testing.assert_allclose(out[0], ref, rtol=1e-4, atol=1e-5)
        c.close()
    finally:
        srv.stop()
