"""YOLOS parity against Hugging Face transformers (the reference demo runs
``hustvl/yolos-small`` through ``YolosForObjectDetection``,
``demos/gpu-sharing-comparison/client/main.py:14-25``).

No checkpoint can be downloaded here: a random-init ``YolosForObjectDetection``
of a small config (the yolos-small layout: no mid position embeddings) is
loaded into :class:`nos_amd.models.yolos.YolosDetector` with
``load_hf_state_dict`` and both run on the CPU in fp32 at two input sizes --
the position embeddings are interpolated (bicubic) in both.  The same weights
then go through the pod-server program path (models/yolos_program.py) too."""
from __future__ import annotations

import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")


def _hf_model():
    cfg = transformers.YolosConfig(hidden_size=128, num_hidden_layers=2, num_attention_heads=2, intermediate_size=256,
                                   image_size=[64, 96], patch_size=16, num_channels=3, num_detection_tokens=10,
                                   num_labels=9, use_mid_position_embeddings=False, layer_norm_eps=1e-12,
                                   hidden_act="gelu", qkv_bias=True)
    torch.manual_seed(0)
    m = transformers.YolosForObjectDetection(cfg).eval()
    with torch.no_grad():  # HF zero-inits the tokens and the embeddings: make every weight non-trivial
        for p in m.parameters():
            p.add_(0.02 * torch.randn_like(p))
    return m


@pytest.mark.parametrize("hw", [(64, 96), (80, 112)])
def test_detector_matches_transformers_yolos(hw):
    from nos_amd.models.yolos import YolosConfig, YolosDetector

    hf = _hf_model()
    ours = YolosDetector(YolosConfig(hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                                     intermediate_size=256, image_size=(64, 96), num_detection_tokens=10,
                                     num_labels=9), backend="torch").eval()
    ours.load_hf_state_dict(hf.state_dict())
    x = torch.randn(2, 3, *hw, generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        ref = hf(pixel_values=x)
        logits, boxes = ours(x)
    assert logits.shape == ref.logits.shape and boxes.shape == ref.pred_boxes.shape
    torch.testing.assert_close(logits, ref.logits, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(boxes, ref.pred_boxes, rtol=1e-5, atol=1e-6)


def test_program_path_matches_transformers_yolos():
    """HF weights -> YolosDetector -> numpy weights -> pod-server program:
    the compiled program (LN folded, epilogues fused) gives HF's outputs."""
    from nos_amd.models.yolos import YolosConfig, YolosDetector
    from nos_amd.models.yolos_program import yolos_program
    from nos_amd.podserver import program as PG

    hf = _hf_model()
    cfg = YolosConfig(hidden_size=128, num_hidden_layers=2, num_attention_heads=2, intermediate_size=256,
                      image_size=(64, 96), num_detection_tokens=10, num_labels=9)
    det = YolosDetector(cfg, backend="torch")
    det.load_hf_state_dict(hf.state_dict())
    weights = {k: v.detach().numpy().copy() for k, v in det.state_dict().items()}
    hw = (80, 112)
    prog = PG.parse(*yolos_program(cfg, weights, hw, "fp32"))
    x = torch.randn(1, 3, *hw, generator=torch.Generator().manual_seed(2))
    with torch.no_grad():
        ref = hf(pixel_values=x)
        out = prog.compile("cpu")(x)
    np.testing.assert_allclose(out[0].numpy(), ref.logits.numpy(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(out[1].numpy(), ref.pred_boxes.numpy(), rtol=1e-4, atol=1e-6)
