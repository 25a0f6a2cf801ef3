"""YOLOS (ViT detector) tenant model -- the workload of the reference's GPU-sharing demo.

The reference benchmarks GPU sharing with pods running ``hustvl/yolos-small``
inference in a loop (``demos/gpu-sharing-comparison/client/main.py:14-25``,
results ``demos/gpu-sharing-comparison/README.md:69-71``).  This module
re-implements that architecture for MI355X:

* every linear layer is one gfx950 MFMA GEMM with a fused epilogue
  (bias, exact GELU, residual add) -- ``nos_gemm_bf16``;
* Q, K and V are one fused projection whose output feeds the flash-style
  attention kernel directly (no head transposes) -- ``nos_attn_fwd_d64``;
* LayerNorm is one bandwidth-bound kernel per call -- ``nos_layernorm_bf16``;
* the whole forward is captured into one HIP graph per tenant
  (:class:`GraphedTenant`), replayed on the tenant's (CU-masked) stream.

Weights are random-initialised (no network, no checkpoints); the architecture
and shapes follow yolos-small: hidden 384, 12 layers, 6 heads, MLP 1536,
16x16 patches, 100 detection tokens, position embeddings for 800x1333
interpolated (bicubic) to the input resolution, 3-layer MLP heads for 92 class
logits and 4 box coordinates.  ``backend="torch"`` runs the same weights
through eager PyTorch ops (hipBLASLt GEMMs + SDPA): the baseline the HIP path
is measured against, and the numerics reference.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .yolos_config import YolosConfig, demo_input_hw, flops_per_image, seq_len


class _Layer(nn.Module):
    def __init__(self, cfg: YolosConfig):
        super().__init__()
        h, m = cfg.hidden_size, cfg.intermediate_size
        self.ln1_w = nn.Parameter(torch.ones(h))
        self.ln1_b = nn.Parameter(torch.zeros(h))
        self.qkv_w = nn.Parameter(torch.empty(3 * h, h))  # rows: [q; k; v], each [H*D]
        self.qkv_b = nn.Parameter(torch.zeros(3 * h))
        self.proj_w = nn.Parameter(torch.empty(h, h))
        self.proj_b = nn.Parameter(torch.zeros(h))
        self.ln2_w = nn.Parameter(torch.ones(h))
        self.ln2_b = nn.Parameter(torch.zeros(h))
        self.fc1_w = nn.Parameter(torch.empty(m, h))
        self.fc1_b = nn.Parameter(torch.zeros(m))
        self.fc2_w = nn.Parameter(torch.empty(h, m))
        self.fc2_b = nn.Parameter(torch.zeros(h))


class YolosDetector(nn.Module):
    """YOLOS object detector (inference)."""

    def __init__(self, cfg: YolosConfig | None = None, backend: str = "native"):
        super().__init__()
        self.cfg = cfg = cfg or YolosConfig.small()
        if cfg.head_dim != 64:
            raise ValueError("nos_amd YOLOS kernels are built for head_dim 64")
        self.backend = backend
        h = cfg.hidden_size
        pd = cfg.num_channels * cfg.patch_size ** 2
        gh0, gw0 = cfg.image_size[0] // cfg.patch_size, cfg.image_size[1] // cfg.patch_size
        self.patch_w = nn.Parameter(torch.empty(h, pd))  # conv 16x16/16 as a GEMM, K = 768
        self.patch_b = nn.Parameter(torch.zeros(h))
        self.cls_token = nn.Parameter(torch.zeros(1, 1, h))
        self.det_tokens = nn.Parameter(torch.zeros(1, cfg.num_detection_tokens, h))
        self.pos_embed = nn.Parameter(torch.zeros(1, 1 + gh0 * gw0 + cfg.num_detection_tokens, h))
        self.layers = nn.ModuleList(_Layer(cfg) for _ in range(cfg.num_hidden_layers))
        self.ln_f_w = nn.Parameter(torch.ones(h))
        self.ln_f_b = nn.Parameter(torch.zeros(h))
        # 3-layer MLP heads (hidden -> hidden -> hidden -> out), ReLU between
        self.cls_head = nn.ParameterList()
        self.box_head = nn.ParameterList()
        for head, out in ((self.cls_head, cfg.num_labels + 1), (self.box_head, 4)):
            for n_in, n_out in ((h, h), (h, h), (h, out)):
                head.append(nn.Parameter(torch.empty(n_out, n_in)))
                head.append(nn.Parameter(torch.zeros(n_out)))
        self._pos_cache: dict[tuple, torch.Tensor] = {}
        self.reset_parameters()

    # ------------------------------------------------------------------ init
    @torch.no_grad()
    def reset_parameters(self, seed: int = 0) -> None:
        g = torch.Generator().manual_seed(seed)
        std = self.cfg.initializer_range
        for name, p in self.named_parameters():
            if p.dim() >= 2 or name.endswith(("cls_token", "det_tokens", "pos_embed")):
                p.copy_(torch.randn(p.shape, generator=g) * std)
        self._pos_cache.clear()

    # ----------------------------------------------------- position embedding
    def interpolated_pos_embed(self, hw: tuple[int, int]) -> torch.Tensor:
        """[1, S, h] position embeddings for input size hw (bicubic, as the
        reference model's InterpolateInitialPositionEmbeddings). A pure function of
        the weights and the input shape, cached per (shape, device, dtype)."""
        key = (hw, self.pos_embed.device, self.pos_embed.dtype, self.pos_embed._version)
        pe = self._pos_cache.get(key)
        if pe is None:
            cfg = self.cfg
            nd = cfg.num_detection_tokens
            p = self.pos_embed.detach().float()
            cls_pe, det_pe, patch_pe = p[:, :1], p[:, -nd:], p[:, 1:-nd]
            gh0, gw0 = cfg.image_size[0] // cfg.patch_size, cfg.image_size[1] // cfg.patch_size
            patch_pe = patch_pe.transpose(1, 2).reshape(1, cfg.hidden_size, gh0, gw0)
            gh, gw = hw[0] // cfg.patch_size, hw[1] // cfg.patch_size
            patch_pe = F.interpolate(patch_pe, size=(gh, gw), mode="bicubic", align_corners=False)
            patch_pe = patch_pe.flatten(2).transpose(1, 2)
            pe = torch.cat([cls_pe, patch_pe, det_pe], dim=1).to(self.pos_embed.dtype).contiguous()
            self._pos_cache = {key: pe}
        return pe

    # --------------------------------------------------------------- forward
    def patchify(self, pixel_values: torch.Tensor) -> torch.Tensor:
        """[B, C, H, W] -> [B, gh*gw, C*p*p] in the conv weight's (c, ky, kx) order."""
        B, C, H, W = pixel_values.shape
        p = self.cfg.patch_size
        gh, gw = H // p, W // p
        x = pixel_values[:, :, : gh * p, : gw * p]
        x = x.reshape(B, C, gh, p, gw, p).permute(0, 2, 4, 1, 3, 5)
        return x.reshape(B, gh * gw, C * p * p)

    def forward(self, pixel_values: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        if self.backend == "torch" or not pixel_values.is_cuda:
            return self._forward_torch(pixel_values)
        return self._forward_native(pixel_values)

    def _embed(self, pixel_values: torch.Tensor, lin) -> torch.Tensor:
        B, _, H, W = pixel_values.shape
        patches = self.patchify(pixel_values.to(self.patch_w.dtype)).contiguous()
        x = lin(patches, self.patch_w, self.patch_b)
        cls = self.cls_token.expand(B, -1, -1)
        det = self.det_tokens.expand(B, -1, -1)
        x = torch.cat([cls, x, det], dim=1)
        return (x + self.interpolated_pos_embed((H, W))).contiguous()

    def _heads(self, x: torch.Tensor, lin) -> tuple[torch.Tensor, torch.Tensor]:
        outs = []
        for head in (self.cls_head, self.box_head):
            y = x
            for i in range(3):
                y = lin(y, head[2 * i], head[2 * i + 1], act="relu" if i < 2 else None)
            outs.append(y)
        return outs[0], outs[1].float().sigmoid()

    @torch.no_grad()
    def folded_weights(self) -> list[dict[str, torch.Tensor]]:
        """Per layer: LayerNorm folded into the following GEMM
        (:func:`nos_amd.ops.fold_layernorm`); recomputed when a weight changes."""
        key = tuple(p._version for p in self.parameters()) + (self.patch_w.device, self.patch_w.dtype)
        if getattr(self, "_folded_key", None) != key:
            out = []
            for L in self.layers:
                qw, qc1, qc2 = ops.fold_layernorm(L.qkv_w, L.qkv_b, L.ln1_w, L.ln1_b)
                fw, fc1, fc2 = ops.fold_layernorm(L.fc1_w, L.fc1_b, L.ln2_w, L.ln2_b)
                out.append({"qkv_w": qw, "qkv_c1": qc1, "qkv_c2": qc2, "fc1_w": fw, "fc1_c1": fc1, "fc1_c2": fc2})
            self._folded = out
            self._folded_key = key
        return self._folded

    def _forward_native(self, pixel_values: torch.Tensor):
        """5 kernels per encoder layer: [LN1+QKV GEMM] [attention]
        [proj GEMM + residual] [LN2+fc1 GEMM + GELU] [fc2 GEMM + residual] --
        the bf16 MFMA kernels for bf16 weights, the exact-fp32 MFMA kernels
        (gemm_f32.hip, attention_f32.hip) for fp32 weights."""
        cfg = self.cfg
        nh = cfg.num_attention_heads
        eps = cfg.layer_norm_eps

        def lin(x, w, b, act=None, residual=None):
            return ops.linear(x.contiguous(), w, b, act=act, residual=residual)

        folded = self.folded_weights()
        h = self._embed(pixel_values, lin)
        # fp32 under x6 math: the QKV projection writes K / V as the attention's
        # bf16x6 / fp16x3 planes directly (no fp32 K/V round trip, no split kernel)
        presplit = ops.ln_qkv_fusable(h)
        # h3 math: attention -> proj and fc1 -> fc2 hand their activations
        # over as the consumer GEMM's fp16 planes (no fp32 round trip, no split pass)
        handoff = presplit and ops.h3_planes_active(attention=True)
        mlp_handoff = h.is_cuda and h.dtype == torch.float32 and ops.h3_planes_active()
        for L, fw in zip(self.layers, folded):
            if presplit:
                a = ops.ln_qkv_attention(h, fw["qkv_w"], fw["qkv_c1"], fw["qkv_c2"], nh, eps=eps, planes_out=handoff)
            else:
                qkv = ops.linear_ln(h, fw["qkv_w"], fw["qkv_c1"], fw["qkv_c2"], eps=eps)
                a = ops.attention_qkv(qkv, nh)
            h = (ops.linear_planes(a, L.proj_w, L.proj_b, residual=h) if handoff
                 else ops.linear(a, L.proj_w, L.proj_b, residual=h))
            if mlp_handoff:
                m = ops.linear_ln_to_planes(h, fw["fc1_w"], fw["fc1_c1"], fw["fc1_c2"], act="gelu", eps=eps)
                h = ops.linear_planes(m, L.fc2_w, L.fc2_b, residual=h)
            else:
                m = ops.linear_ln(h, fw["fc1_w"], fw["fc1_c1"], fw["fc1_c2"], act="gelu", eps=eps)
                h = ops.linear(m, L.fc2_w, L.fc2_b, residual=h)
        det = h[:, -cfg.num_detection_tokens:, :].contiguous()
        if det.dtype == torch.float32:  # 100 rows: not worth a kernel of its own in fp32
            y = F.layer_norm(det, (cfg.hidden_size,), self.ln_f_w, self.ln_f_b, eps)
        else:
            y, _ = ops.layernorm(det, self.ln_f_w, self.ln_f_b, eps)
        return self._heads(y, lin)

    def _forward_torch(self, pixel_values: torch.Tensor, native_attention: bool = False):
        """Eager PyTorch (numerics reference): torch GEMMs + SDPA.
        ``native_attention`` swaps in the gfx950 fp32 MFMA flash attention
        (``nos_attn_fwd_f32_d64``) on the fused QKV output, to test attention
        alone; the fp32 pods themselves run :meth:`_forward_native` (the
        exact-fp32 MFMA GEMMs of ``gemm_f32.hip`` + that attention)."""
        cfg = self.cfg
        nh, hd = cfg.num_attention_heads, cfg.head_dim

        def lin(x, w, b, act=None, residual=None):
            y = F.linear(x, w, b)
            if act == "gelu":
                y = F.gelu(y)
            elif act == "relu":
                y = F.relu(y)
            return y if residual is None else y + residual

        h = self._embed(pixel_values, lin)
        B, S, hs = h.shape
        eps = cfg.layer_norm_eps
        for L in self.layers:
            y = F.layer_norm(h, (hs,), L.ln1_w, L.ln1_b, eps)
            qkv = F.linear(y, L.qkv_w, L.qkv_b)
            if native_attention:
                a = ops.attention_qkv(qkv, nh)
            else:
                q, k, v = (t.transpose(1, 2) for t in qkv.view(B, S, 3, nh, hd).unbind(2))
                a = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, S, hs)
            h = F.linear(a, L.proj_w, L.proj_b) + h
            y = F.layer_norm(h, (hs,), L.ln2_w, L.ln2_b, eps)
            h = F.linear(F.gelu(F.linear(y, L.fc1_w, L.fc1_b)), L.fc2_w, L.fc2_b) + h
        y = F.layer_norm(h, (hs,), self.ln_f_w, self.ln_f_b, eps)
        det = y[:, -cfg.num_detection_tokens:, :]
        return self._heads(det, lin)

    @torch.no_grad()
    def load_numpy(self, weights: dict) -> None:
        """Load numpy weights named like this module's parameters (the
        pod-server program's weights, models/yolos_program.py)."""
        self.load_state_dict({k: torch.from_numpy(v) for k, v in weights.items()}, strict=True)
        self._pos_cache.clear()

    # ------------------------------------------------------ HF weight import
    @torch.no_grad()
    def load_hf_state_dict(self, sd: dict[str, torch.Tensor]) -> None:
        """Import a transformers YolosForObjectDetection state dict (parity tests)."""
        def g(k):
            return sd[k].to(self.patch_w.dtype)

        self.patch_w.copy_(g("vit.embeddings.patch_embeddings.projection.weight").reshape(self.patch_w.shape))
        self.patch_b.copy_(g("vit.embeddings.patch_embeddings.projection.bias"))
        self.cls_token.copy_(g("vit.embeddings.cls_token"))
        self.det_tokens.copy_(g("vit.embeddings.detection_tokens"))
        self.pos_embed.copy_(g("vit.embeddings.position_embeddings"))
        for i, L in enumerate(self.layers):
            p = f"vit.encoder.layer.{i}."
            L.ln1_w.copy_(g(p + "layernorm_before.weight"))
            L.ln1_b.copy_(g(p + "layernorm_before.bias"))
            L.qkv_w.copy_(torch.cat([g(p + f"attention.attention.{n}.weight") for n in ("query", "key", "value")]))
            L.qkv_b.copy_(torch.cat([g(p + f"attention.attention.{n}.bias") for n in ("query", "key", "value")]))
            L.proj_w.copy_(g(p + "attention.output.dense.weight"))
            L.proj_b.copy_(g(p + "attention.output.dense.bias"))
            L.ln2_w.copy_(g(p + "layernorm_after.weight"))
            L.ln2_b.copy_(g(p + "layernorm_after.bias"))
            L.fc1_w.copy_(g(p + "intermediate.dense.weight"))
            L.fc1_b.copy_(g(p + "intermediate.dense.bias"))
            L.fc2_w.copy_(g(p + "output.dense.weight"))
            L.fc2_b.copy_(g(p + "output.dense.bias"))
        self.ln_f_w.copy_(g("vit.layernorm.weight"))
        self.ln_f_b.copy_(g("vit.layernorm.bias"))
        for head, name in ((self.cls_head, "class_labels_classifier"), (self.box_head, "bbox_predictor")):
            for i in range(3):
                head[2 * i].copy_(g(f"{name}.layers.{i}.weight"))
                head[2 * i + 1].copy_(g(f"{name}.layers.{i}.bias"))
        self._pos_cache.clear()


@dataclass
class GraphedTenant:
    """One tenant "pod": a model instance + static input, captured into a HIP
    graph on its own stream (the stream carries the tenant's CU mask)."""

    model: YolosDetector
    stream: torch.cuda.Stream
    pixel_values: torch.Tensor
    graph: torch.cuda.CUDAGraph | None = None
    outputs: tuple = field(default_factory=tuple)

    def capture(self, warmup: int = 2, capture_error_mode: str = "global", pool=None, light: bool = False) -> None:
        """``capture_error_mode="thread_local"`` when other threads keep
        launching while this one captures (the pod server's lanes); ``pool``
        shares another graph's memory pool (graphs never replayed at once).
        ``light``: capture on this stream only, without the device-wide
        synchronize, ``gc.collect()`` and ``empty_cache()`` that
        ``torch.cuda.graph`` runs first -- in the pod server those waited for
        every lane's in-flight replays and walked the whole Python heap per
        capture (the warm-ups are synchronised on this stream instead)."""
        with torch.cuda.stream(self.stream):
            for _ in range(warmup):
                self.outputs = self.model(self.pixel_values)
        self.stream.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        if light:
            with torch.cuda.stream(self.stream):
                if pool is None:
                    self.graph.capture_begin(capture_error_mode=capture_error_mode)
                else:
                    self.graph.capture_begin(pool, capture_error_mode=capture_error_mode)
                try:
                    self.outputs = self.model(self.pixel_values)
                finally:
                    self.graph.capture_end()
        else:
            with torch.cuda.graph(self.graph, pool=pool, stream=self.stream, capture_error_mode=capture_error_mode):
                self.outputs = self.model(self.pixel_values)
        self.stream.synchronize()

    def launch(self) -> None:
        with torch.cuda.stream(self.stream):
            if self.graph is not None:
                self.graph.replay()
            else:
                self.outputs = self.model(self.pixel_values)


def make_demo_input(cfg: YolosConfig, batch: int = 1, device="cpu", dtype=torch.bfloat16,
                    hw: tuple[int, int] | None = None, seed: int = 0) -> torch.Tensor:
    """Synthetic normalised image batch of the demo's shape (no dataset access)."""
    hw = hw or demo_input_hw()
    g = torch.Generator().manual_seed(seed)
    x = torch.randn((batch, cfg.num_channels, *hw), generator=g)
    return x.to(device=device, dtype=dtype)


__all__ = ["YolosConfig", "YolosDetector", "GraphedTenant", "make_demo_input", "demo_input_hw",
           "flops_per_image", "seq_len", "math"]
