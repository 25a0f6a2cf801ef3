"""YOLOS configuration and shape helpers, free of torch (pod-server client
pods build their program with numpy only: models/yolos_program.py)."""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class YolosConfig:
    hidden_size: int = 384
    num_hidden_layers: int = 12
    num_attention_heads: int = 6
    intermediate_size: int = 1536
    patch_size: int = 16
    num_channels: int = 3
    image_size: tuple[int, int] = (800, 1333)
    num_detection_tokens: int = 100
    num_labels: int = 91
    layer_norm_eps: float = 1e-12
    initializer_range: float = 0.02

    @classmethod
    def small(cls) -> "YolosConfig":
        return cls()

    @classmethod
    def tiny(cls) -> "YolosConfig":
        return cls(hidden_size=192, num_attention_heads=3, intermediate_size=768, image_size=(800, 1333))

    @classmethod
    def test(cls) -> "YolosConfig":
        """Small config for CPU tests (head_dim stays 64)."""
        return cls(hidden_size=128, num_hidden_layers=2, num_attention_heads=2, intermediate_size=256,
                   image_size=(64, 96), num_detection_tokens=10, num_labels=9)

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads


def demo_input_hw() -> tuple[int, int]:
    """Input size of the reference demo: COCO val2017 #39769 (640x480) resized by
    YolosImageProcessor to shortest edge 800 (longest <= 1333) -> 800 x 1066."""
    h, w = 480, 640
    s = 800 / min(h, w)
    nh, nw = int(round(h * s)), int(w * s)
    if max(nh, nw) > 1333:
        s = 1333 / max(h, w)
        nh, nw = int(h * s), int(w * s)
    return nh, nw


def flops_per_image(cfg: YolosConfig, hw: tuple[int, int]) -> float:
    """Multiply-add FLOPs of one forward at input size hw (matmuls + attention)."""
    gh, gw = hw[0] // cfg.patch_size, hw[1] // cfg.patch_size
    S = 1 + gh * gw + cfg.num_detection_tokens
    h, m = cfg.hidden_size, cfg.intermediate_size
    per_layer = 2 * S * h * (3 * h) + 2 * S * h * h + 2 * 2 * S * h * m + 2 * 2 * S * S * h
    patch = 2 * gh * gw * (cfg.num_channels * cfg.patch_size ** 2) * h
    heads = 2 * cfg.num_detection_tokens * (4 * h * h + h * (cfg.num_labels + 1) + h * 4)
    return float(cfg.num_hidden_layers * per_layer + patch + heads)


def seq_len(cfg: YolosConfig, hw: tuple[int, int]) -> int:
    return 1 + (hw[0] // cfg.patch_size) * (hw[1] // cfg.patch_size) + cfg.num_detection_tokens


__all__ = ["YolosConfig", "demo_input_hw", "flops_per_image", "seq_len"]
