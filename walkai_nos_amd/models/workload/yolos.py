"""YOLOS-small: the fractional-GPU benchmark workload.

The reference's only published performance numbers come from its GPU-sharing demo, in which every
Pod runs ``hustvl/yolos-small`` inference at batch 1 on one COCO image in a loop
(``demos/gpu-sharing-comparison/client/main.py:6-35``).  This module is an
independent implementation of that architecture (ViT-S/16 encoder with 100 detection tokens and
DETR-style MLP heads) built for the MI355X inference path:

* fp32 end to end (the reference demo runs fp32 PyTorch; no precision is given up): on the GPU every
  product runs in the x3 format — fp32 operands split exactly into three bf16 planes, six bf16
  MFMAs per block, fp32-accurate (``ops/kernels.py: set_fp32_matmul``); ``f32`` mode uses the
  f32-input MFMA instead;
* the interpolated position embeddings are computed once per input resolution and cached (the
  upstream implementation re-interpolates on every forward);
* the hot ops dispatch to hand-written HIP kernels (:mod:`walkai_nos_amd.ops.kernels`) on the GPU:
  LayerNorm that emits x3 planes, x3 GEMMs with bias / exact GELU / residuals fused into the store
  (the QKV projection leaves as fp32, which the x3 flash attention splits in-kernel), and the
  stream-K x3 flash attention; the detection heads (100 tokens) stay on ``torch`` / hipBLASLt;
* ``load_hf_state_dict`` maps a ``transformers`` ``YolosForObjectDetection`` state dict onto this
  module, which is how numerical parity is tested
  (``tests/test_infra.py::test_yolos_matches_transformers_reference``) — there is no network, so
  weights are random-init of the same architecture.

Config (hustvl/yolos-small): hidden 384, 12 layers, 6 heads, MLP 1536, patch 16, 100 detection
tokens, pre-training image size 800x1333, 91 COCO labels (+1 "no object").  The demo's 640x480
image is resized by the YOLOS processor to 800x1066 (shortest edge 800) -> 50x66 patches ->
3401 tokens.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ...ops import kernels as K


@dataclass
class YolosConfig:
    hidden_size: int = 384
    num_layers: int = 12
    num_heads: int = 6
    intermediate_size: int = 1536
    patch_size: int = 16
    num_channels: int = 3
    num_detection_tokens: int = 100
    image_size: Tuple[int, int] = (800, 1333)
    num_labels: int = 91
    layer_norm_eps: float = 1e-12
    use_mid_position_embeddings: bool = False

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_heads


#: the demo's input after YolosImageProcessor (640x480 COCO image -> shortest edge 800)
DEMO_INPUT_HW = (800, 1066)


class _Block(nn.Module):
    def __init__(self, c: YolosConfig):
        super().__init__()
        d, f = c.hidden_size, c.intermediate_size
        self.c = c
        self.ln1 = nn.LayerNorm(d, eps=c.layer_norm_eps)
        self.qkv = nn.Linear(d, 3 * d)            # fused q|k|v projection
        self.proj = nn.Linear(d, d)
        self.ln2 = nn.LayerNorm(d, eps=c.layer_norm_eps)
        self.fc1 = nn.Linear(d, f)
        self.fc2 = nn.Linear(f, d)

    def forward_x3(self, x: torch.Tensor, mid: Optional[torch.Tensor], h3: Optional[torch.Tensor],
                   next_ln: Optional[nn.LayerNorm]) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        """The x3 path with the LayerNorms folded into the producing step: ``h3`` is LN1(x) as planes
        when the previous block already made it; the projection step returns x and LN2(x), the fc2
        step x and ``next_ln``(x) (the next block's LN1) — each either the fused-epilogue GEMM + a
        LayerNorm kernel or a split-K GEMM + one combine-and-LayerNorm kernel, whichever is faster
        on the slice (``ops.gemm.linear_residual_ln_x3``)."""
        H, Dh = self.c.num_heads, self.c.head_dim
        eps = self.c.layer_norm_eps
        if h3 is None:
            h3 = K.layernorm_x3(x, self.ln1.weight, self.ln1.bias, eps)
        if K.attention_input_f32():
            qkv = K.linear_x3(h3, self.qkv.weight, self.qkv.bias)
            if K.attn_proj_fusable(H, Dh):
                # attention partials -> one merge + projection + residual + LN2 kernel
                x, h3 = K.attention_proj_ln_x3f(qkv, H, Dh, 1.0 / math.sqrt(Dh), self.proj.weight, self.proj.bias,
                                                x, (self.ln2.weight, self.ln2.bias, eps))
            else:
                o3 = K.attention_qkv_x3f(qkv, H, Dh, 1.0 / math.sqrt(Dh))
                x, h3 = K.linear_residual_ln_x3(o3, self.proj.weight, self.proj.bias, x,
                                                ln=(self.ln2.weight, self.ln2.bias, eps))
        else:
            qkv3 = K.linear_x3(h3, self.qkv.weight, self.qkv.bias, out_x3=True)
            o3 = K.attention_qkv_x3(qkv3, H, Dh, 1.0 / math.sqrt(Dh))
            x, h3 = K.linear_residual_ln_x3(o3, self.proj.weight, self.proj.bias, x,
                                            ln=(self.ln2.weight, self.ln2.bias, eps))
        f3 = K.linear_x3(h3, self.fc1.weight, self.fc1.bias, gelu=True, out_x3=True)
        nl = (next_ln.weight, next_ln.bias, next_ln.eps) if next_ln is not None else None
        return K.linear_residual_ln_x3(f3, self.fc2.weight, self.fc2.bias, x, residual2=mid, ln=nl)

    def forward(self, x: torch.Tensor, mid: Optional[torch.Tensor] = None) -> torch.Tensor:
        B, T, D = x.shape
        H, Dh = self.c.num_heads, self.c.head_dim
        if K.x3_active(x):
            # every fp32 product on the bf16 matrix cores in x3 form: activations leave their
            # producer as three exact bf16 planes; the residual stream stays fp32
            h3 = K.layernorm_x3(x, self.ln1.weight, self.ln1.bias, self.c.layer_norm_eps)
            if K.attention_input_f32():
                # QKV leaves the GEMM as fp32 (4 B per element); attention splits it in-kernel
                qkv = K.linear_x3(h3, self.qkv.weight, self.qkv.bias)
                o3 = K.attention_qkv_x3f(qkv, H, Dh, 1.0 / math.sqrt(Dh))
            else:
                qkv3 = K.linear_x3(h3, self.qkv.weight, self.qkv.bias, out_x3=True)
                o3 = K.attention_qkv_x3(qkv3, H, Dh, 1.0 / math.sqrt(Dh))
            x = K.linear_x3(o3, self.proj.weight, self.proj.bias, residual=x)
            h3 = K.layernorm_x3(x, self.ln2.weight, self.ln2.bias, self.c.layer_norm_eps)
            f3 = K.linear_x3(h3, self.fc1.weight, self.fc1.bias, gelu=True, out_x3=True)
            return K.linear_x3(f3, self.fc2.weight, self.fc2.bias, residual=x, residual2=mid)
        h = K.layernorm(x, self.ln1.weight, self.ln1.bias, self.c.layer_norm_eps)
        qkv = K.linear(h, self.qkv.weight, self.qkv.bias)                  # [B, T, 3D]
        o = K.attention_qkv(qkv, H, Dh, 1.0 / math.sqrt(Dh))               # [B, T, D]
        x = K.linear_residual(o, self.proj.weight, self.proj.bias, x)      # x + o @ Wp^T + bp
        h = K.layernorm(x, self.ln2.weight, self.ln2.bias, self.c.layer_norm_eps)
        h = K.linear_gelu(h, self.fc1.weight, self.fc1.bias)               # gelu(h @ W1^T + b1)
        return K.linear_residual(h, self.fc2.weight, self.fc2.bias, x, mid)   # (+ mid pos-embed, fused)


class _MLPHead(nn.Module):
    def __init__(self, d_in: int, d_hidden: int, d_out: int, n_layers: int = 3):
        super().__init__()
        dims = [d_in] + [d_hidden] * (n_layers - 1)
        self.layers = nn.ModuleList(nn.Linear(a, b) for a, b in zip(dims, dims[1:] + [d_out]))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        for i, l in enumerate(self.layers):
            x = l(x)
            if i < len(self.layers) - 1:
                x = F.relu(x)
        return x


class YolosSmall(nn.Module):
    def __init__(self, c: Optional[YolosConfig] = None):
        super().__init__()
        c = c or YolosConfig()
        self.c = c
        d = c.hidden_size
        gh, gw = c.image_size[0] // c.patch_size, c.image_size[1] // c.patch_size
        self.cls_token = nn.Parameter(torch.zeros(1, 1, d))
        self.det_tokens = nn.Parameter(torch.zeros(1, c.num_detection_tokens, d))
        self.pos_embed = nn.Parameter(torch.zeros(1, 1 + gh * gw + c.num_detection_tokens, d))
        self.patch = nn.Conv2d(c.num_channels, d, kernel_size=c.patch_size, stride=c.patch_size)
        self.mid_pos_embed = (nn.Parameter(torch.zeros(c.num_layers - 1, 1, 1 + gh * gw + c.num_detection_tokens, d))
                              if c.use_mid_position_embeddings else None)
        self.blocks = nn.ModuleList(_Block(c) for _ in range(c.num_layers))
        self.ln_f = nn.LayerNorm(d, eps=c.layer_norm_eps)
        self.cls_head = _MLPHead(d, d, c.num_labels + 1)
        self.box_head = _MLPHead(d, d, 4)
        self._pos_cache: Dict[Tuple[int, int, str, int], torch.Tensor] = {}
        self.reset_parameters()

    def reset_parameters(self, seed: int = 0) -> None:
        g = torch.Generator().manual_seed(seed)
        with torch.no_grad():
            for p in self.parameters():
                if p.dim() >= 2:
                    p.copy_(torch.randn(p.shape, generator=g) * 0.02)
                else:
                    p.zero_()
            for m in self.modules():
                if isinstance(m, nn.LayerNorm):
                    m.weight.fill_(1.0)

    # -- position embeddings ---------------------------------------------------------------
    def _interp(self, pe: torch.Tensor, hw: Tuple[int, int]) -> torch.Tensor:
        c = self.c
        nd = c.num_detection_tokens
        gh, gw = c.image_size[0] // c.patch_size, c.image_size[1] // c.patch_size
        cls_pe, patch_pe, det_pe = pe[..., :1, :], pe[..., 1:-nd, :], pe[..., -nd:, :]
        lead = patch_pe.shape[:-2]
        patch_pe = patch_pe.reshape(-1, gh, gw, c.hidden_size).permute(0, 3, 1, 2)
        nh, nw = hw[0] // c.patch_size, hw[1] // c.patch_size
        patch_pe = F.interpolate(patch_pe, size=(nh, nw), mode="bicubic", align_corners=False)
        patch_pe = patch_pe.flatten(2).transpose(1, 2).reshape(*lead, nh * nw, c.hidden_size)
        return torch.cat((cls_pe, patch_pe, det_pe), dim=-2)

    def position_embeddings(self, hw: Tuple[int, int]) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        key = (hw[0], hw[1], str(self.pos_embed.device), self.pos_embed._version)
        if key not in self._pos_cache:
            with torch.no_grad():
                pe = self._interp(self.pos_embed, hw).contiguous()
                mid = self._interp(self.mid_pos_embed, hw).contiguous() if self.mid_pos_embed is not None else None
            self._pos_cache.clear()
            self._pos_cache[key] = (pe, mid)
        return self._pos_cache[key]

    def invalidate_cache(self) -> None:
        self._pos_cache.clear()
        self._tok_key = None

    # -- forward -------------------------------------------------------------------------
    def forward(self, pixels: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        B, _, Hh, Ww = pixels.shape
        pe, mid = self.position_embeddings((Hh, Ww))
        nd = self.c.num_detection_tokens
        hip = B == 1 and pixels.is_cuda and K.get_backend() == "hip"
        if hip:
            # one copy of the token template (class/detection token rows already + pos), then the
            # patch rows written straight into it by the GEMM (bias + pos fused)
            P = (Hh // self.c.patch_size) * (Ww // self.c.patch_size)
            x = self.token_template((Hh, Ww)).clone()
            K.patch_embed(pixels, self.patch.weight, self.patch.bias, self.c.patch_size, pe[0, 1:1 + P],
                          out=x[0, 1:1 + P])
        else:
            xp = K.patch_embed(pixels, self.patch.weight, self.patch.bias, self.c.patch_size)   # [B, P, D]
            x = torch.cat((self.cls_token.expand(B, -1, -1), xp, self.det_tokens.expand(B, -1, -1)), dim=1) + pe
        if K.x3_active(x):
            h3 = None
            for i, blk in enumerate(self.blocks):
                nxt = self.blocks[i + 1].ln1 if i + 1 < len(self.blocks) else None
                x, h3 = blk.forward_x3(x, mid[i] if mid is not None and i < self.c.num_layers - 1 else None, h3, nxt)
        else:
            for i, blk in enumerate(self.blocks):
                x = blk(x, mid[i] if mid is not None and i < self.c.num_layers - 1 else None)
        det = x[:, -self.c.num_detection_tokens:, :]
        if hip and x.is_contiguous() and self.heads_fusable():
            # final LayerNorm + both MLP heads in three launches (csrc/head.hip)
            logits, boxes = K.detection_heads(det[0], self.ln_f, self.cls_head.layers, self.box_head.layers)
            return logits[None], boxes[None]
        det = K.layernorm(det.contiguous(), self.ln_f.weight, self.ln_f.bias, self.c.layer_norm_eps)
        return self.cls_head(det), torch.sigmoid(self.box_head(det))

    def heads_fusable(self) -> bool:
        """Both heads are 3-layer MLPs of one shape with rows of at most 384 (a multiple of 4) —
        what the fused kernel stages in LDS (``csrc/head.hip``); otherwise the module path runs."""
        ch, bh = self.cls_head.layers, self.box_head.layers
        d, hid = self.c.hidden_size, ch[0].weight.shape[0]
        return (len(ch) == 3 and len(bh) == 3 and ch[0].weight.shape == bh[0].weight.shape
                and ch[1].weight.shape == bh[1].weight.shape and d <= 384 and hid <= 384
                and d % 4 == 0 and hid % 4 == 0)

    def token_template(self, hw: Tuple[int, int]) -> torch.Tensor:
        """[1, T, D]: the class-token row + its position embedding, zero patch rows, the detection-token
        rows + theirs — cached per parameter versions (every forward copies it once)."""
        key = (hw, str(self.pos_embed.device), self.pos_embed._version, self.cls_token._version,
               self.det_tokens._version)
        if getattr(self, "_tok_key", None) != key:
            pe, _ = self.position_embeddings(hw)
            nd = self.c.num_detection_tokens
            with torch.no_grad():
                t = torch.zeros_like(pe)
                t[:, :1] = self.cls_token + pe[:, :1]
                t[:, -nd:] = self.det_tokens + pe[:, -nd:]
            self._tok, self._tok_key = t, key
        return self._tok

    def flops_per_inference(self, hw: Tuple[int, int] = DEMO_INPUT_HW) -> float:
        c = self.c
        T = 1 + (hw[0] // c.patch_size) * (hw[1] // c.patch_size) + c.num_detection_tokens
        d, f = c.hidden_size, c.intermediate_size
        per_layer = 2 * T * (3 * d * d + d * d + 2 * d * f) + 4 * T * T * d
        patch = 2 * (T - 1 - c.num_detection_tokens) * d * c.num_channels * c.patch_size ** 2
        return float(c.num_layers * per_layer + patch)

    # -- weights ------------------------------------------------------------------------
    def load_hf_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        """Map ``transformers`` YolosForObjectDetection weights onto this module."""
        own: Dict[str, torch.Tensor] = {
            "cls_token": sd["vit.embeddings.cls_token"],
            "det_tokens": sd["vit.embeddings.detection_tokens"],
            "pos_embed": sd["vit.embeddings.position_embeddings"],
            "patch.weight": sd["vit.embeddings.patch_embeddings.projection.weight"],
            "patch.bias": sd["vit.embeddings.patch_embeddings.projection.bias"],
            "ln_f.weight": sd["vit.layernorm.weight"],
            "ln_f.bias": sd["vit.layernorm.bias"],
        }
        if self.mid_pos_embed is not None:
            own["mid_pos_embed"] = sd["vit.encoder.mid_position_embeddings"]
        for i in range(self.c.num_layers):
            p = f"vit.encoder.layer.{i}."
            a = p + "attention."
            own[f"blocks.{i}.qkv.weight"] = torch.cat([sd[a + f"attention.{n}.weight"] for n in ("query", "key", "value")])
            own[f"blocks.{i}.qkv.bias"] = torch.cat([sd[a + f"attention.{n}.bias"] for n in ("query", "key", "value")])
            own[f"blocks.{i}.proj.weight"] = sd[a + "output.dense.weight"]
            own[f"blocks.{i}.proj.bias"] = sd[a + "output.dense.bias"]
            own[f"blocks.{i}.ln1.weight"] = sd[p + "layernorm_before.weight"]
            own[f"blocks.{i}.ln1.bias"] = sd[p + "layernorm_before.bias"]
            own[f"blocks.{i}.ln2.weight"] = sd[p + "layernorm_after.weight"]
            own[f"blocks.{i}.ln2.bias"] = sd[p + "layernorm_after.bias"]
            own[f"blocks.{i}.fc1.weight"] = sd[p + "intermediate.dense.weight"]
            own[f"blocks.{i}.fc1.bias"] = sd[p + "intermediate.dense.bias"]
            own[f"blocks.{i}.fc2.weight"] = sd[p + "output.dense.weight"]
            own[f"blocks.{i}.fc2.bias"] = sd[p + "output.dense.bias"]
        for head, hf in (("cls_head", "class_labels_classifier"), ("box_head", "bbox_predictor")):
            for j in range(3):
                own[f"{head}.layers.{j}.weight"] = sd[f"{hf}.layers.{j}.weight"]
                own[f"{head}.layers.{j}.bias"] = sd[f"{hf}.layers.{j}.bias"]
        missing, unexpected = self.load_state_dict(own, strict=True), None
        del missing, unexpected
        self.invalidate_cache()


def demo_input(batch: int = 1, hw: Tuple[int, int] = DEMO_INPUT_HW, device: str = "cpu", seed: int = 0) -> torch.Tensor:
    """A normalised image tensor of the demo's processed shape (synthetic; no dataset access)."""
    g = torch.Generator().manual_seed(seed)
    return torch.randn(batch, 3, hw[0], hw[1], generator=g).to(device)
