"""Depth-Anything-V2 (DINOv2 ViT backbone + DPT-style neck + relative-depth head) on MI355X.

This is the model the reference actually loads: `load_model("depth-anything-v2")`,
backend/app.py:78-82, hub name depth-anything/Depth-Anything-V2-Small-hf, which
`process_with_depth_anything` runs at :109-116. Weights use the transformers
`DepthAnythingForDepthEstimation` state-dict layout (transformers 5.15,
modeling_depth_anything.py plus dinov2/modeling_dinov2.py), so a local safetensors
export of the hub checkpoint loads unchanged. Every block runs on the gfx950
kernels of libi2pc.so: bf16 operands, fp32 accumulation, fp32 residual stream.

  embeddings   patch rows (K = 3*14*14 padded to 640 with zeros) -> GEMM + bias +
               position table; the table is bicubically interpolated once per grid
               when the grid differs from the checkpoint's (Dinov2Embeddings.
               interpolate_pos_encoding); CLS row = cls + pos[0]
  encoder x L  LN -> QKV -> attention -> O -> +res -> LN -> FC1+GELU -> FC2 -> +res.
               LayerScale is folded into the O / FC2 weight rows and biases
               (lambda * (W x + b) = (lambda W) x + lambda b)          modeling_dinov2.py Dinov2Layer
               With dpt.LN_FOLD the two LNs are folded through QKV / FC1: O and FC2
               write the residual's bf16 copy and 32-column row partials in their
               epilogue, QKV / FC1 apply (rstd, -rstd*mean) in theirs (_encoder_folded)
  features     backbone LayerNorm of the hidden states after layers out_indices
  reassemble   drop CLS (GEMM row remap) -> 1x1 projection -> ConvT(4)/ConvT(2)/
               id/3x3 s2 conv                                       modeling_depth_anything.py:31-93
  neck convs   3x3, no bias, to `fusion` channels                   :217-262
  fusion x 4   residual units as conv GEMMs; resize to the next map's size
               (align_corners=True); the 1x1 projection is evaluated before the
               resize (linear maps whose bilinear weights sum to one commute)  :96-206
  head         3x3 conv -> resize to (14*gh, 14*gw) align_corners=True -> 3x3 conv
               + ReLU -> 1x1 conv + ReLU (relative depth, max_depth 1)          :265-308

Channel counts that are not multiples of the kernels' granules (48 and 96 in the
neck, 32 in the head) are zero-padded in the packed weights (exact: padded
channels carry zeros and meet zero weights).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

from . import dpt, ops
from .dpt import _pack_conv
from .preprocess import patch_pitch

# LayerNorm-fold partial width (columns per (mean, M2) chunk; dpt.LN_FOLD switches the fold)
LN_CHUNK = 32


@dataclass(frozen=True)
class DASpec:
    name: str
    hidden: int
    layers: int
    heads: int
    mlp: int
    out_indices: tuple          # 1-based stage numbers (stage k = output of layer k)
    neck: tuple = (48, 96, 192, 384)
    fusion: int = 64
    head_hidden: int = 32
    factors: tuple = (4, 2, 1, 0.5)
    patch: int = 14
    image: int = 518            # checkpoint grid = image // patch
    eps: float = 1e-6
    family: str = "depth-anything"

    @property
    def grid(self) -> int:
        return self.image // self.patch

    def hf_config_kwargs(self) -> dict:
        return dict(backbone_config=dict(model_type="dinov2", hidden_size=self.hidden,
                                         num_hidden_layers=self.layers, num_attention_heads=self.heads,
                                         mlp_ratio=self.mlp // self.hidden, patch_size=self.patch,
                                         image_size=self.image, layer_norm_eps=self.eps,
                                         out_indices=list(self.out_indices), apply_layernorm=True,
                                         reshape_hidden_states=False),
                    patch_size=self.patch, reassemble_hidden_size=self.hidden,
                    neck_hidden_sizes=list(self.neck), reassemble_factors=list(self.factors),
                    fusion_hidden_size=self.fusion, head_hidden_size=self.head_hidden,
                    depth_estimation_type="relative")

    def sizes(self, gh: int, gw: int):
        """Spatial size of each reassembled map for a gh x gw patch grid."""
        out = []
        for fac in self.factors:
            if fac > 1:
                out.append((gh * int(fac), gw * int(fac)))
            elif fac == 1:
                out.append((gh, gw))
            else:
                s = int(1 / fac)
                out.append(((gh - 1) // s + 1, (gw - 1) // s + 1))
        return out

    def flops_per_image(self, gh: int = None, gw: int = None) -> float:
        """Algorithmic FLOPs (2 x MAC, un-padded channel counts; + 4*T^2*d*L attention)."""
        gh = gh or self.grid
        gw = gw or self.grid
        D, T, n = self.hidden, gh * gw + 1, gh * gw
        F = self.fusion
        f = 2.0 * n * 3 * self.patch ** 2 * D
        f += self.layers * (2.0 * T * (4 * D * D + 2 * D * self.mlp) + 4.0 * T * T * D)
        sizes = self.sizes(gh, gw)
        for c, fac, (h, w) in zip(self.neck, self.factors, sizes):
            f += 2.0 * n * D * c
            if fac > 1:
                f += 2.0 * n * c * c * fac * fac
            elif fac < 1:
                f += 2.0 * h * w * 9 * c * c
            f += 2.0 * h * w * 9 * c * F
        for j, (h, w) in enumerate(reversed(sizes)):
            f += (1 if j == 0 else 2) * 2 * 2.0 * h * w * 9 * F * F + 2.0 * h * w * F * F
        h, w = 2 * sizes[0][0], 2 * sizes[0][1]
        f += 2.0 * h * w * 9 * F * (F // 2)
        H, W = gh * self.patch, gw * self.patch
        f += 2.0 * H * W * 9 * (F // 2) * self.head_hidden + 2.0 * H * W * self.head_hidden
        return f


DA_V2_SMALL = DASpec("depth-anything-v2-small", hidden=384, layers=12, heads=6, mlp=1536,
                     out_indices=(9, 10, 11, 12))
# a small member of the family for fast parity tests (real neck/head widths, short backbone)
DA_TINY = DASpec("depth-anything-tiny", hidden=128, layers=4, heads=2, mlp=512, out_indices=(1, 2, 3, 4),
                 image=168)


def state_dict_keys(spec: DASpec) -> dict:
    """name -> shape of every tensor DepthAnythingForDepthEstimation(config) holds."""
    D, P, T = spec.hidden, spec.patch, spec.grid ** 2 + 1
    k = {"backbone.embeddings.cls_token": (1, 1, D), "backbone.embeddings.mask_token": (1, D),
         "backbone.embeddings.position_embeddings": (1, T, D),
         "backbone.embeddings.patch_embeddings.projection.weight": (D, 3, P, P),
         "backbone.embeddings.patch_embeddings.projection.bias": (D,),
         "backbone.layernorm.weight": (D,), "backbone.layernorm.bias": (D,)}
    for i in range(spec.layers):
        p = f"backbone.encoder.layer.{i}."
        for n in ("norm1", "norm2"):
            k[p + n + ".weight"] = (D,)
            k[p + n + ".bias"] = (D,)
        for n in ("query", "key", "value"):
            k[p + f"attention.attention.{n}.weight"] = (D, D)
            k[p + f"attention.attention.{n}.bias"] = (D,)
        k[p + "attention.output.dense.weight"] = (D, D)
        k[p + "attention.output.dense.bias"] = (D,)
        k[p + "layer_scale1.lambda1"] = (D,)
        k[p + "layer_scale2.lambda1"] = (D,)
        k[p + "mlp.fc1.weight"] = (spec.mlp, D)
        k[p + "mlp.fc1.bias"] = (spec.mlp,)
        k[p + "mlp.fc2.weight"] = (D, spec.mlp)
        k[p + "mlp.fc2.bias"] = (D,)
    F = spec.fusion
    for i, (c, fac) in enumerate(zip(spec.neck, spec.factors)):
        p = f"neck.reassemble_stage.layers.{i}."
        k[p + "projection.weight"] = (c, D, 1, 1)
        k[p + "projection.bias"] = (c,)
        if fac > 1:
            k[p + "resize.weight"] = (c, c, int(fac), int(fac))
            k[p + "resize.bias"] = (c,)
        elif fac < 1:
            k[p + "resize.weight"] = (c, c, 3, 3)
            k[p + "resize.bias"] = (c,)
        k[f"neck.convs.{i}.weight"] = (F, c, 3, 3)
        p = f"neck.fusion_stage.layers.{i}."
        k[p + "projection.weight"] = (F, F, 1, 1)
        k[p + "projection.bias"] = (F,)
        for r in ("residual_layer1", "residual_layer2"):
            for cv in ("convolution1", "convolution2"):
                k[p + f"{r}.{cv}.weight"] = (F, F, 3, 3)
                k[p + f"{r}.{cv}.bias"] = (F,)
    k["head.conv1.weight"] = (F // 2, F, 3, 3)
    k["head.conv1.bias"] = (F // 2,)
    k["head.conv2.weight"] = (spec.head_hidden, F // 2, 3, 3)
    k["head.conv2.bias"] = (spec.head_hidden,)
    k["head.conv3.weight"] = (1, spec.head_hidden, 1, 1)
    k["head.conv3.bias"] = (1,)
    return k


def synthetic_state_dict(spec: DASpec, seed: int = 0):
    """Deterministic random weights (the hub checkpoint is a remote name, unavailable offline)."""
    import torch
    g = torch.Generator(device="cpu").manual_seed(seed)
    sd = {}
    for name, shape in state_dict_keys(spec).items():
        if name.endswith("cls_token") or name.endswith("mask_token"):
            t = 0.5 * torch.randn(shape, generator=g)
        elif name.endswith("position_embeddings"):
            t = 0.1 * torch.randn(shape, generator=g)
        elif name.endswith("lambda1"):
            t = 0.5 + 0.5 * torch.rand(shape, generator=g)
        elif ("norm" in name) and name.endswith("weight"):
            t = 1.0 + 0.1 * torch.randn(shape, generator=g)
        elif name == "head.conv3.bias":
            t = torch.full(shape, 2.0)
        elif name.endswith("bias"):
            t = 0.02 * torch.randn(shape, generator=g)
        elif name == "head.conv3.weight":
            t = 0.5 * torch.randn(shape, generator=g) / math.sqrt(shape[1])
        elif "reassemble" in name and name.endswith("resize.weight") and shape[2] in (2, 4):
            t = torch.randn(shape, generator=g) / math.sqrt(shape[0])
        else:
            fan_in = int(torch.tensor(shape[1:]).prod())
            t = torch.randn(shape, generator=g) / math.sqrt(fan_in)
        sd[name] = t.float()
    return sd


def _pad_to(n: int, q: int) -> int:
    return (n + q - 1) // q * q


class DepthAnythingModel:
    """bf16 Depth-Anything forward on MI355X.

    `forward(patches, B, gh, gw)` -> depth fp32 [B, 14*gh, 14*gw]; `patches` are the
    preprocess 'patches' rows (pitch 640)."""

    def __init__(self, spec: DASpec, state_dict: dict, device):
        import torch
        self.spec = spec
        self.device = torch.device(device)
        self._bufs = {}
        self._pos = {}
        dev = self.device
        sd = {k: v.detach().to(torch.float32).cpu() for k, v in state_dict.items()}
        self._sd_pos = sd["backbone.embeddings.position_embeddings"][0]
        bf = lambda t: t.to(torch.bfloat16).contiguous().to(dev)     # noqa: E731
        f32 = lambda t: t.to(torch.float32).contiguous().to(dev)     # noqa: E731
        D, P = spec.hidden, spec.patch
        kp = patch_pitch(P)
        pe = sd["backbone.embeddings.patch_embeddings.projection.weight"].reshape(D, 3 * P * P)
        self.w_pe = bf(torch.nn.functional.pad(pe, (0, kp - 3 * P * P)))
        self.b_pe = f32(sd["backbone.embeddings.patch_embeddings.projection.bias"])
        self.cls = f32(sd["backbone.embeddings.cls_token"].reshape(D))
        self.pos0 = f32(self._sd_pos[0])
        self.layers = []
        for i in range(spec.layers):
            p = f"backbone.encoder.layer.{i}."
            q = [sd[p + f"attention.attention.{n}.weight"] for n in ("query", "key", "value")]
            qb = [sd[p + f"attention.attention.{n}.bias"] for n in ("query", "key", "value")]
            # softmax scale * log2(e) folded into the Q rows (fp32, before the bf16 rounding): the QKV GEMM
            # writes Q in the exp2 domain that attention(..., q_log2=True) takes
            wq, bq = ops.fold_q_scale(torch.cat(q, 0), torch.cat(qb, 0), 1.0 / math.sqrt(spec.hidden // spec.heads))
            q, qb = [wq], [bq]
            l1 = sd[p + "layer_scale1.lambda1"]
            l2 = sd[p + "layer_scale2.lambda1"]
            L = dict(
                ln1_g=f32(sd[p + "norm1.weight"]), ln1_b=f32(sd[p + "norm1.bias"]),
                w_qkv=bf(torch.cat(q, 0)), b_qkv=f32(torch.cat(qb, 0)),
                w_o=bf(sd[p + "attention.output.dense.weight"] * l1[:, None]),
                b_o=f32(sd[p + "attention.output.dense.bias"] * l1),
                ln2_g=f32(sd[p + "norm2.weight"]), ln2_b=f32(sd[p + "norm2.bias"]),
                w_1=bf(sd[p + "mlp.fc1.weight"]), b_1=f32(sd[p + "mlp.fc1.bias"]),
                w_2=bf(sd[p + "mlp.fc2.weight"] * l2[:, None]), b_2=f32(sd[p + "mlp.fc2.bias"] * l2),
            )
            # the LN-folded forms of QKV (norm1) and FC1 (norm2), as in dpt.py
            wf, cs, bfold = ops.ln_fold_weights(torch.cat(q, 0), torch.cat(qb, 0), sd[p + "norm1.weight"],
                                                sd[p + "norm1.bias"])
            L.update(w_qkv_f=wf.to(dev), s_qkv=cs.to(dev), b_qkv_f=bfold.to(dev))
            wf, cs, bfold = ops.ln_fold_weights(sd[p + "mlp.fc1.weight"], sd[p + "mlp.fc1.bias"], sd[p + "norm2.weight"],
                                                sd[p + "norm2.bias"])
            L.update(w_1_f=wf.to(dev), s_1=cs.to(dev), b_1_f=bfold.to(dev))
            self.layers.append(L)
        self.ln_g = f32(sd["backbone.layernorm.weight"])
        self.ln_b = f32(sd["backbone.layernorm.bias"])
        F = spec.fusion
        self.stages = []
        for i, (c, fac) in enumerate(zip(spec.neck, spec.factors)):
            p = f"neck.reassemble_stage.layers.{i}."
            cp = _pad_to(c, 64)                      # padded channel count of this map
            wp = torch.zeros(cp, D)
            wp[:c] = sd[p + "projection.weight"].reshape(c, D)
            bp = torch.zeros(cp)
            bp[:c] = sd[p + "projection.bias"]
            wn = torch.zeros(F, cp, 3, 3)
            wn[:, :c] = sd[f"neck.convs.{i}.weight"]
            st = dict(c=cp, fac=fac, w_proj=bf(wp), b_proj=f32(bp), w_neck=_pack_conv(wn, torch).to(dev))
            if fac > 1:
                s = int(fac)
                w = torch.zeros(cp, cp, s, s)                            # [Ci, Co, s, s]
                w[:c, :c] = sd[p + "resize.weight"]
                b = torch.zeros(cp)
                b[:c] = sd[p + "resize.bias"]
                st["w_rs"] = bf(w.permute(2, 3, 1, 0).reshape(s * s * cp, cp))
                st["b_rs"] = f32(b.repeat(s * s))
            elif fac < 1:
                w = torch.zeros(cp, cp, 3, 3)
                w[:c, :c] = sd[p + "resize.weight"]
                b = torch.zeros(cp)
                b[:c] = sd[p + "resize.bias"]
                st["w_rs"] = _pack_conv(w, torch).to(dev)
                st["b_rs"] = f32(b)
                st["stride"] = int(round(1 / fac))
            self.stages.append(st)
        self.fusion = []
        for i in range(len(spec.neck)):
            p = f"neck.fusion_stage.layers.{i}."
            fl = dict(w_proj=bf(sd[p + "projection.weight"].reshape(F, F)), b_proj=f32(sd[p + "projection.bias"]))
            for r in ("residual_layer1", "residual_layer2"):
                for cv in ("convolution1", "convolution2"):
                    fl[f"{r}.{cv}.w"] = _pack_conv(sd[p + f"{r}.{cv}.weight"], torch).to(dev)
                    fl[f"{r}.{cv}.b"] = f32(sd[p + f"{r}.{cv}.bias"])
            self.fusion.append(fl)
        h1 = F // 2
        self.h1p = _pad_to(h1, 64)
        w1 = torch.zeros(self.h1p, F, 3, 3)
        w1[:h1] = sd["head.conv1.weight"]
        b1 = torch.zeros(self.h1p)
        b1[:h1] = sd["head.conv1.bias"]
        self.w_h1, self.b_h1 = _pack_conv(w1, torch).to(dev), f32(b1)
        hh = spec.head_hidden
        w2 = torch.zeros(hh, self.h1p, 3, 3)
        w2[:, :h1] = sd["head.conv2.weight"]
        self.w_h2, self.b_h2 = _pack_conv(w2, torch).to(dev), f32(sd["head.conv2.bias"])
        self.w_h3 = f32(sd["head.conv3.weight"].reshape(hh))
        self.b_h3 = float(sd["head.conv3.bias"].reshape(()).item())

    # ------------------------------------------------------------------ per-grid state
    def pos_table(self, gh: int, gw: int):
        """Patch rows of the position table for a gh x gw grid (Dinov2Embeddings.interpolate_pos_encoding)."""
        import torch
        key = (gh, gw)
        if key not in self._pos:
            g0 = self.spec.grid
            tab = self._sd_pos[1:]
            if (gh, gw) != (g0, g0):
                D = tab.shape[1]
                t = tab.reshape(1, g0, g0, D).permute(0, 3, 1, 2)
                t = torch.nn.functional.interpolate(t, size=(gh, gw), mode="bicubic", align_corners=False)
                tab = t.permute(0, 2, 3, 1).reshape(gh * gw, D)
            self._pos[key] = tab.to(torch.float32).contiguous().to(self.device)
        return self._pos[key]

    def buffers(self, B: int, gh: int, gw: int) -> dict:
        import torch
        key = (B, gh, gw)
        if key in self._bufs:
            return self._bufs[key]
        s, dev = self.spec, self.device
        D = s.hidden
        M = B * (gh * gw + 1)
        e = lambda shape, dt=torch.bfloat16: torch.empty(shape, dtype=dt, device=dev)   # noqa: E731
        b = dict(x=e((M, D), torch.float32), ln=e((M, D)), qkv=e((M, 3 * D)), att=e((M, D)), mlp=e((M, s.mlp)),
                 hs=[e((M, D)) for _ in s.out_indices],
                 part=e((M, D // LN_CHUNK, 2), torch.float32), rs=e((M, 2), torch.float32), shift=e((M,), torch.float32),
                 shift2=e((M,), torch.float32))
        b["ln_fold"] = dpt.LN_FOLD and D % LN_CHUNK == 0 and self._ln_fold_ok(b, M)
        self._bufs[key] = b
        return b

    def _ln_fold_ok(self, b, M) -> bool:
        """Whether libi2pc.so takes the LN-folded calls at this size (i2pc_gemm_kernel_name is
        "invalid" for a descriptor i2pc_gemm would reject)."""
        L, D = self.layers[0], self.spec.hidden

        def name(x, w, out, **kw):
            d = ops.GemmDesc()
            d.a, d.lda, d.m, d.n, d.k = x.data_ptr(), x.stride(0), M, w.shape[0], w.shape[1]
            d.w, d.ldw, d.c, d.ldc = w.data_ptr(), w.stride(0), out.data_ptr(), out.stride(0)
            d.c_f32 = int(out.element_size() == 4)
            for k, v in kw.items():
                setattr(d, k, v)
            return ops.gemm_kernel_label(d)
        consumer = dict(ln_rows=b["rs"].data_ptr(), col_sum=L["s_qkv"].data_ptr(), bias=L["b_qkv_f"].data_ptr())
        producer = dict(res=b["x"].data_ptr(), res_f32=1, ldr=D, ln_part=b["part"].data_ptr(), ln_chunk=LN_CHUNK,
                        c_bf16=b["ln"].data_ptr(), ldc_bf16=D, ln_shift=b["shift"].data_ptr())
        names = [name(b["ln"], L["w_qkv_f"], b["qkv"], **consumer),
                 name(b["ln"], L["w_1_f"], b["mlp"], **dict(consumer, col_sum=L["s_1"].data_ptr(), act=1)),
                 name(b["att"], L["w_o"], b["x"], **producer),
                 name(b["mlp"], L["w_2"], b["x"], **producer)]
        if dpt.BF16_STREAM:   # bf16-output producers (layer 0's attention-out reads the fp32 embeddings)
            stream = dict(res=b["ln"].data_ptr(), res_f32=0, ldr=D, ln_part=b["part"].data_ptr(), ln_chunk=LN_CHUNK,
                          ln_shift=b["shift"].data_ptr(), res_shift=b["shift2"].data_ptr())
            names += [name(b["att"], L["w_o"], b["ln"], **dict(producer, c_bf16=0, ldc_bf16=0)),
                      name(b["att"], L["w_o"], b["ln"], **stream),
                      name(b["mlp"], L["w_2"], b["ln"], **stream)]
        return "invalid" not in names

    # ------------------------------------------------------------------ forward
    def forward(self, patches, B: int, gh: int = None, gw: int = None):
        s = self.spec
        gh = gh or s.grid
        gw = gw or s.grid
        D = s.hidden
        np_, T = gh * gw, gh * gw + 1
        buf = self.buffers(B, gh, gw)
        x = buf["x"]
        ops.linear(patches, self.w_pe, bias=self.b_pe, table=self.pos_table(gh, gw), table_rows=np_, out=x,
                   out_map=(np_, T, 1), rows=B * np_)
        ops.cls_pos(self.cls, self.pos0, x, B, T, D)
        scale = 1.0 / math.sqrt(D // s.heads)
        hs_i = 0
        if buf["ln_fold"]:
            self._encoder_folded(buf, B, T, scale)
        for i, L in enumerate(self.layers if not buf["ln_fold"] else ()):
            ln = ops.layernorm(x, L["ln1_g"], L["ln1_b"], s.eps, out=buf["ln"])
            qkv = ops.linear(ln, L["w_qkv"], bias=L["b_qkv"], out=buf["qkv"])
            att = ops.attention(qkv, B, T, s.heads, scale, out=buf["att"], q_log2=True)
            ops.linear(att, L["w_o"], bias=L["b_o"], res=x, out=x)
            ln = ops.layernorm(x, L["ln2_g"], L["ln2_b"], s.eps, out=buf["ln"])
            h = ops.linear(ln, L["w_1"], bias=L["b_1"], act="gelu", out=buf["mlp"])
            ops.linear(h, L["w_2"], bias=L["b_2"], res=x, out=x)
            if (i + 1) in s.out_indices:
                ops.layernorm(x, self.ln_g, self.ln_b, s.eps, out=buf["hs"][hs_i])    # backbone LayerNorm
                hs_i += 1
        feats = [self._reassemble(j, buf["hs"][j], B, gh, gw) for j in range(len(self.stages))]
        hidden = None
        rev = list(reversed(feats))
        for j, feat in enumerate(rev):
            size = tuple(rev[j + 1].shape[1:3]) if j + 1 < len(rev) else None
            hidden = self._fuse(self.fusion[j], feat, hidden, size)
        t = ops.conv2d(hidden, self.w_h1, bias=self.b_h1)
        H, W = gh * s.patch, gw * s.patch
        if dpt.FUSED_HEAD and s.head_hidden == 32:
            return ops.head_upconv(t, H, W, self.w_h2, self.b_h2, self.w_h3, self.b_h3, cin=_pad_to(s.fusion // 2, 32))
        u = ops.resize_bilinear(t, H, W, align_corners=True)
        t2 = ops.conv2d(u, self.w_h2, bias=self.b_h2, act="relu")
        return ops.head_out(t2, self.w_h3, self.b_h3)

    __call__ = forward

    def _encoder_folded(self, buf, B, T, scale):
        """The encoder with norm1 / norm2 folded through QKV / FC1 (include/i2pc.h "LayerNorm
        fold"): attention-out and FC2 write the residual's bf16 copy (minus the previous LayerNorm's
        row mean) and 32-column (mean, M2) partials in their epilogue (the 384-column outputs run on
        384 x 192 tiles whose 96-column wave tiles hold no whole 64-column chunk); ln_rowstats turns
        them into (rstd, -rstd * mean) rows the next QKV / FC1 epilogue applies.  The backbone
        LayerNorm of the kept hidden states stays a LayerNorm kernel on the fp32 rows."""
        s = self.spec
        x = buf["x"]
        nl = len(self.layers)
        hs_i = 0
        a_in = None
        if dpt.BF16_STREAM:
            return self._encoder_stream(buf, B, T, scale)
        for i, L in enumerate(self.layers):
            if a_in is None:      # layer 0: norm1 of the embeddings (its row means: the first shift)
                ln = ops.layernorm(x, L["ln1_g"], L["ln1_b"], s.eps, out=buf["ln"], mean_out=buf["shift"])
                qkv = ops.linear(ln, L["w_qkv"], bias=L["b_qkv"], out=buf["qkv"])
            else:
                qkv = ops.linear(a_in, L["w_qkv_f"], bias=L["b_qkv_f"], ln_rows=buf["rs"], col_sum=L["s_qkv"],
                                 out=buf["qkv"])
            att = ops.attention(qkv, B, T, s.heads, scale, out=buf["att"], q_log2=True)
            ops.linear(att, L["w_o"], bias=L["b_o"], res=x, out=x, ln_part=buf["part"], out_bf16=buf["ln"],
                       ln_shift=buf["shift"], ln_chunk=LN_CHUNK)
            ops.ln_rowstats(buf["part"], s.eps, out=buf["rs"], shift_in=buf["shift"], shift_out=buf["shift"],
                            chunk=LN_CHUNK)
            h = ops.linear(buf["ln"], L["w_1_f"], bias=L["b_1_f"], act="gelu", ln_rows=buf["rs"], col_sum=L["s_1"],
                           out=buf["mlp"])
            if i + 1 < nl:
                # FC2 + residual; its shifted bf16 copy and partials feed the next layer's QKV
                ops.linear(h, L["w_2"], bias=L["b_2"], res=x, out=x, ln_part=buf["part"], out_bf16=buf["ln"],
                           ln_shift=buf["shift"], ln_chunk=LN_CHUNK)
                ops.ln_rowstats(buf["part"], s.eps, out=buf["rs"], shift_in=buf["shift"], shift_out=buf["shift"],
                                chunk=LN_CHUNK)
                a_in = buf["ln"]
            else:
                ops.linear(h, L["w_2"], bias=L["b_2"], res=x, out=x)
            if (i + 1) in s.out_indices:
                ops.layernorm(x, self.ln_g, self.ln_b, s.eps, out=buf["hs"][hs_i])    # backbone LayerNorm
                hs_i += 1

    def _encoder_stream(self, buf, B, T, scale):
        """The folded encoder on the shifted bf16 residual stream (dpt.BF16_STREAM; i2pc.h "bf16
        residual stream"): attention-out and FC2 read buf["ln"] (stored relative to one shift buffer)
        and write it back in place relative to the other, the latest LayerNorm mean; the backbone
        LayerNorm of a kept hidden state is applied from FC2's row statistics (ops.ln_apply) instead of
        a LayerNorm pass over an fp32 stream."""
        s = self.spec
        sh0, sh1 = buf["shift"], buf["shift2"]
        hs_i = 0
        res, rsh = buf["x"], None          # layer 0: the residual is the fp32 embeddings
        for i, L in enumerate(self.layers):
            if i == 0:                     # norm1 of the embeddings (its row means: the first shift)
                ln = ops.layernorm(buf["x"], L["ln1_g"], L["ln1_b"], s.eps, out=buf["ln"], mean_out=sh0)
                qkv = ops.linear(ln, L["w_qkv"], bias=L["b_qkv"], out=buf["qkv"])
            else:
                qkv = ops.linear(buf["ln"], L["w_qkv_f"], bias=L["b_qkv_f"], ln_rows=buf["rs"], col_sum=L["s_qkv"],
                                 out=buf["qkv"])
            att = ops.attention(qkv, B, T, s.heads, scale, out=buf["att"], q_log2=True)
            ops.linear(att, L["w_o"], bias=L["b_o"], res=res, res_shift=rsh, out=buf["ln"], ln_part=buf["part"],
                       ln_shift=sh0, ln_chunk=LN_CHUNK)
            ops.ln_rowstats(buf["part"], s.eps, out=buf["rs"], shift_in=sh0, shift_out=sh1, chunk=LN_CHUNK)
            h = ops.linear(buf["ln"], L["w_1_f"], bias=L["b_1_f"], act="gelu", ln_rows=buf["rs"], col_sum=L["s_1"],
                           out=buf["mlp"])
            ops.linear(h, L["w_2"], bias=L["b_2"], res=buf["ln"], res_shift=sh0, out=buf["ln"], ln_part=buf["part"],
                       ln_shift=sh1, ln_chunk=LN_CHUNK)
            ops.ln_rowstats(buf["part"], s.eps, out=buf["rs"], shift_in=sh1, shift_out=sh0, chunk=LN_CHUNK)
            res, rsh = buf["ln"], sh1
            if (i + 1) in s.out_indices:   # backbone LayerNorm (same eps) from the same row statistics
                ops.ln_apply(buf["ln"], buf["rs"], self.ln_g, self.ln_b, out=buf["hs"][hs_i])
                hs_i += 1

    def _reassemble(self, j, hs, B, gh, gw):
        st = self.stages[j]
        np_, T = gh * gw, gh * gw + 1
        c = st["c"]
        proj = ops.linear(hs, st["w_proj"], bias=st["b_proj"], rows=B * np_, a_map=(np_, T, 1)).view(B, gh, gw, c)
        fac = st["fac"]
        if fac > 1:
            r = ops.conv_transpose(proj, st["w_rs"], st["b_rs"], int(fac))
        elif fac == 1:
            r = proj
        else:
            r = ops.conv2d(proj, st["w_rs"], bias=st["b_rs"], k=3, stride=st["stride"], pad=1)
        return ops.conv2d(r, st["w_neck"])

    def _fuse(self, fl, feat, hidden, size):
        if hidden is None:
            h = feat
        else:
            if tuple(hidden.shape) != tuple(feat.shape):
                # modeling_depth_anything.py:159-163: the incoming feature is resized to the fused map
                # (not reached for the grids the reassemble sizes produce)
                feat = ops.resize_bilinear(feat, hidden.shape[1], hidden.shape[2], align_corners=False)
            t = ops.conv2d(feat, fl["residual_layer1.convolution1.w"], bias=fl["residual_layer1.convolution1.b"],
                           relu_in=True, act="relu")
            h = ops.conv2d(t, fl["residual_layer1.convolution2.w"], bias=fl["residual_layer1.convolution2.b"],
                           res=feat, res2=hidden)
        t = ops.conv2d(h, fl["residual_layer2.convolution1.w"], bias=fl["residual_layer2.convolution1.b"],
                       relu_in=True, act="relu")
        h2 = ops.conv2d(t, fl["residual_layer2.convolution2.w"], bias=fl["residual_layer2.convolution2.b"], res=h)
        B, H, W, F = h2.shape
        p = ops.linear(h2.view(B * H * W, F), fl["w_proj"], bias=fl["b_proj"]).view(B, H, W, F)
        if size is None:
            size = (2 * H, 2 * W)
        return ops.resize_bilinear(p, size[0], size[1], align_corners=True)
