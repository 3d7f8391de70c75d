"""DPT-Hybrid depth network (BiT-ResNet-50 stem + ViT-B/16 + DPT neck/head) on MI355X,
bf16 or MX fp8 (BASELINE.json configs[4]).

Weights are taken in the transformers `DPTForDepthEstimation(is_hybrid=True)` state-dict
layout (transformers 5.15 modeling_dpt.py:89-182, 456-557; modeling_bit.py), so a local
safetensors export of Intel/dpt-hybrid-midas loads unchanged.  The reference backend reaches
this family through the same model-loading branch as its Depth-Anything model
(backend/app.py:78-82, AutoModelForDepthEstimation.from_pretrained).

  BiT stem     7x7/2 SAME conv (weight-standardised at load) -> GroupNorm + ReLU -> 3x3/2
               max pool -> bottleneck stages [3, 4, 9] (1x1 -> GN/ReLU -> 3x3 -> GN/ReLU ->
               1x1 -> GN, + (GN(1x1 downsample) | identity), ReLU)          modeling_bit.py:226-547
  embeddings   1x1 projection 1024 -> 768 of stage 3 + CLS + position table  modeling_dpt.py:159-182
  encoder x 12 as DPT-Large (ViT-B: d 768, 12 heads, MLP 3072)              modeling_dpt.py:101-254
  neck         stages 0 / 1 = BiT stage 1 / 2 maps (identity reassemble); stages 2 / 3 =
               readout "project" of layers 8 / 11, 1x1 projection, identity / 3x3 s2 conv;
               3x3 convs to 256                                               modeling_dpt.py:484-557
  fusion, head as DPT-Large                                                   modeling_dpt.py:390-509, 679-716

Precision.  dtype="fp8": every linear layer of the encoder and the readout, and every 3x3
conv of the neck, the fusion stage and the head's first conv run on the MX fp8 engine
(i2pc_gemm_fp8: e4m3fn operands, one E8M0 scale per 32 k, fp32 accumulation).  Weights are
quantised once at load (ops.quantize_mx); activations are quantised by their producer
(LayerNorm, the FC1 / conv1 / readout epilogues) or by one i2pc_quant_fp8 pass.  The BiT stem
(~9 % of the FLOPs, GroupNorm-bound), the embedding projection, the attention core, the
readout's CLS half, the fusion 1x1 projections and the fused head tail stay bf16.
dtype="bf16": the DPT-Large kernels throughout.  `bf16_points` keeps named groups of an fp8
model in bf16 (FP8_POINTS: "qkv", "o", "fc1", "fc2" of every encoder layer, "readout", "neck",
"fusion", "head"): the per-point ablation of tests/test_dpt_hybrid_gpu.py, and the mixed default
DEFAULT_BF16_POINTS chosen from it.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

from . import ops
from .dpt import DPTDepthModel, DPTSpec, _pack_conv


# quantisation points of the fp8 path (groups of GEMMs whose inputs and weights are MX fp8)
FP8_POINTS = ("qkv", "o", "fc1", "fc2", "readout", "neck", "fusion", "head")
# groups the fp8 model keeps in bf16 by default (chosen from the per-point ablation)
DEFAULT_BF16_POINTS = ("qkv", "fc2")


@dataclass(frozen=True)
class HybridSpec(DPTSpec):
    bit_depths: tuple = (3, 4, 9)
    bit_widths: tuple = (256, 512, 1024)
    stem: int = 64
    groups: int = 32

    def hf_config_kwargs(self) -> dict:
        kw = super().hf_config_kwargs()
        kw.update(is_hybrid=True, backbone_featmap_shape=[1, self.bit_widths[-1], self.grid, self.grid],
                  neck_ignore_stages=[0, 1],
                  backbone_config=dict(depths=list(self.bit_depths), embedding_dynamic_padding=True,
                                       global_padding="same", hidden_sizes=list(self.bit_widths) + [2 * self.bit_widths[-1]],
                                       layer_type="bottleneck", out_features=["stage1", "stage2", "stage3"],
                                       embedding_size=self.stem, num_groups=self.groups))
        return kw

    def bit_layers(self):
        """(stage, layer, in_ch, mid, out_ch, stride) of every bottleneck (BitStage, modeling_bit.py:473-545)."""
        out = []
        c = self.stem
        for s, (d, w) in enumerate(zip(self.bit_depths, self.bit_widths)):
            for l in range(d):
                out.append((s, l, c, w // 4, w, (1 if s == 0 else 2) if l == 0 else 1))
                c = w
        return out

    def flops_per_image(self) -> float:
        """2 x MAC of every conv / linear + 4 T^2 d L attention, as this module computes them."""
        g, D, T, F = self.grid, self.hidden, self.grid ** 2 + 1, self.fusion
        s = self.image // 2
        f = 2.0 * s * s * 49 * 3 * self.stem                               # stem conv
        s //= 2
        for st, l, ci, mid, co, stride in self.bit_layers():
            so = s // stride
            f += 2.0 * s * s * ci * mid + 2.0 * so * so * 9 * mid * mid + 2.0 * so * so * mid * co
            if l == 0:
                f += 2.0 * so * so * ci * co
            s = so
        f += 2.0 * g * g * self.bit_widths[-1] * D                          # embedding projection
        f += self.layers * 2.0 * T * (4 * D * D + 2 * D * self.mlp)        # QKV, O, FC1, FC2
        f += self.layers * 4.0 * T * T * D                                 # attention
        sizes = [4 * g, 2 * g, g, (g + 1) // 2]
        chans = [self.bit_widths[0], self.bit_widths[1], self.neck[2], self.neck[3]]
        for j in (2, 3):
            c = self.neck[j]
            f += 2.0 * g * g * D * D + 2.0 * D * D + 2.0 * g * g * D * c    # readout + projection
            if self.factors[j] < 1:
                f += 2.0 * sizes[3] ** 2 * 9 * c * c
        for c, sz in zip(chans, sizes):
            f += 2.0 * sz * sz * 9 * c * F                                 # neck convs
        for j, sz in enumerate(reversed(sizes)):
            units = 1 if j == 0 else 2
            f += units * 2 * 2.0 * sz * sz * 9 * F * F + 2.0 * sz * sz * F * F
        s = 2 * sizes[0]
        f += 2.0 * s * s * 9 * F * (F // 2)
        f += 2.0 * (2 * s) ** 2 * 9 * (F // 2) * 32 + 2.0 * (2 * s) ** 2 * 32
        return f


DPT_HYBRID = HybridSpec("dpt-hybrid", hidden=768, layers=12, heads=12, mlp=3072, patch=16, image=384,
                        out_indices=(2, 5, 8, 11), neck=(256, 512, 768, 768), fusion=256, factors=(1, 1, 1, 0.5),
                        family="dpt-hybrid")
# a small member of the same family for fast parity tests (BiT widths kept: the stem's
# GroupNorm / conv shapes are the real ones; one bottleneck per stage)
DPT_HYBRID_TINY = HybridSpec("dpt-hybrid-tiny", hidden=256, layers=4, heads=4, mlp=512, patch=16, image=128,
                             out_indices=(0, 1, 2, 3), neck=(256, 512, 256, 256), fusion=256, factors=(1, 1, 1, 0.5),
                             family="dpt-hybrid", bit_depths=(1, 1, 1))


def state_dict_keys(spec: HybridSpec) -> dict:
    """name -> shape of every tensor DPTForDepthEstimation(hybrid config) holds."""
    D, T, F = spec.hidden, spec.grid ** 2 + 1, spec.fusion
    p = "dpt.embeddings.backbone.bit."
    k = {"dpt.embeddings.cls_token": (1, 1, D), "dpt.embeddings.position_embeddings": (1, T, D),
         p + "embedder.convolution.weight": (spec.stem, 3, 7, 7),
         p + "embedder.norm.weight": (spec.stem,), p + "embedder.norm.bias": (spec.stem,)}
    for s, l, ci, mid, co, stride in spec.bit_layers():
        q = p + f"encoder.stages.{s}.layers.{l}."
        if l == 0:
            k[q + "downsample.conv.weight"] = (co, ci, 1, 1)
            k[q + "downsample.norm.weight"] = (co,)
            k[q + "downsample.norm.bias"] = (co,)
        for n, shape in (("1", (mid, ci, 1, 1)), ("2", (mid, mid, 3, 3)), ("3", (co, mid, 1, 1))):
            k[q + f"conv{n}.weight"] = shape
            k[q + f"norm{n}.weight"] = (shape[0],)
            k[q + f"norm{n}.bias"] = (shape[0],)
    k["dpt.embeddings.projection.weight"] = (D, spec.bit_widths[-1], 1, 1)
    k["dpt.embeddings.projection.bias"] = (D,)
    for i in range(spec.layers):
        q = f"dpt.encoder.layer.{i}."
        for n in ("query", "key", "value"):
            k[q + f"attention.attention.{n}.weight"] = (D, D)
            k[q + f"attention.attention.{n}.bias"] = (D,)
        k[q + "attention.output.dense.weight"] = (D, D)
        k[q + "attention.output.dense.bias"] = (D,)
        k[q + "intermediate.dense.weight"] = (spec.mlp, D)
        k[q + "intermediate.dense.bias"] = (spec.mlp,)
        k[q + "output.dense.weight"] = (D, spec.mlp)
        k[q + "output.dense.bias"] = (D,)
        for n in ("layernorm_before", "layernorm_after"):
            k[q + n + ".weight"] = (D,)
            k[q + n + ".bias"] = (D,)
    k["dpt.layernorm.weight"] = (D,)
    k["dpt.layernorm.bias"] = (D,)
    for i in (2, 3):
        c = spec.neck[i]
        q = f"neck.reassemble_stage.layers.{i}."
        k[q + "projection.weight"] = (c, D, 1, 1)
        k[q + "projection.bias"] = (c,)
        if spec.factors[i] < 1:
            k[q + "resize.weight"] = (c, c, 3, 3)
            k[q + "resize.bias"] = (c,)
        k[f"neck.reassemble_stage.readout_projects.{i}.0.weight"] = (D, 2 * D)
        k[f"neck.reassemble_stage.readout_projects.{i}.0.bias"] = (D,)
    for i, c in enumerate(spec.neck):
        k[f"neck.convs.{i}.weight"] = (F, c, 3, 3)
        q = f"neck.fusion_stage.layers.{i}."
        k[q + "projection.weight"] = (F, F, 1, 1)
        k[q + "projection.bias"] = (F,)
        for r in ("residual_layer1", "residual_layer2"):
            for cv in ("convolution1", "convolution2"):
                k[q + f"{r}.{cv}.weight"] = (F, F, 3, 3)
                k[q + f"{r}.{cv}.bias"] = (F,)
    k["head.head.0.weight"] = (F // 2, F, 3, 3)
    k["head.head.0.bias"] = (F // 2,)
    k["head.head.2.weight"] = (32, F // 2, 3, 3)
    k["head.head.2.bias"] = (32,)
    k["head.head.4.weight"] = (1, 32, 1, 1)
    k["head.head.4.bias"] = (1,)
    return k


def synthetic_state_dict(spec: HybridSpec, seed: int = 0):
    """Deterministic random weights (no pretrained checkpoint offline): fan-in-scaled normal
    convs / linears, GroupNorm / LayerNorm gains near 1, a positive final bias.

    The last GroupNorm of every BiT residual branch (norm3) gets gain ~0.2, as trained
    ResNets have (BiT / timm recipes zero-initialise that gain): with unit gains a random
    16-block BiT is chaotic -- transformers' own bf16 forward then differs from its fp32
    forward by 11 % (relative L2 of the depth, stage 3 maps 39 %; measured r02), which would
    make every low-precision parity check meaningless.  With 0.2 it is 1 %."""
    import torch
    g = torch.Generator(device="cpu").manual_seed(seed)
    sd = {}
    for name, shape in state_dict_keys(spec).items():
        if name.endswith("cls_token"):
            t = 0.5 * torch.randn(shape, generator=g)
        elif name.endswith("position_embeddings"):
            t = 0.1 * torch.randn(shape, generator=g)
        elif name.endswith("norm3.weight"):
            t = 0.2 * (1.0 + 0.1 * torch.randn(shape, generator=g))
        elif ("norm" in name) and name.endswith("weight") and len(shape) == 1:
            t = 1.0 + 0.1 * torch.randn(shape, generator=g)
        elif name == "head.head.4.bias":
            t = torch.full(shape, 2.0)
        elif name.endswith("bias"):
            t = 0.02 * torch.randn(shape, generator=g)
        elif name == "head.head.4.weight":
            t = 0.5 * torch.randn(shape, generator=g) / math.sqrt(32)
        else:
            fan_in = int(torch.tensor(shape[1:]).prod())
            t = torch.randn(shape, generator=g) / math.sqrt(fan_in)
        sd[name] = t.float()
    return sd


def standardize(w, eps=1e-8):
    """WeightStandardizedConv2d's weight transform (modeling_bit.py:118-127), the same torch call."""
    import torch
    return torch.nn.functional.batch_norm(w.reshape(1, w.shape[0], -1), None, None, training=True, momentum=0.0,
                                          eps=eps).reshape_as(w)


class DPTHybridModel(DPTDepthModel):
    """DPT-Hybrid forward on MI355X.  `forward(pixels, B)` with pixels fp32 NCHW [B, 3, 384, 384]
    (Preprocessor layout "nchw") -> depth fp32 [B, 384, 384]."""

    input_layout = "nchw"

    def __init__(self, spec: HybridSpec, state_dict: dict, device, dtype: str = "fp8", bf16_points=None):
        import torch
        if dtype not in ("bf16", "fp8"):
            raise ValueError(f"dtype must be 'bf16' or 'fp8', got {dtype!r}")
        self.spec, self.dtype = spec, dtype
        self.bf16_points = frozenset(DEFAULT_BF16_POINTS if bf16_points is None else bf16_points)
        if not self.bf16_points <= set(FP8_POINTS):
            raise ValueError(f"unknown bf16 points {sorted(self.bf16_points - set(FP8_POINTS))}; known: {FP8_POINTS}")
        self.device = torch.device(device)
        self._bufs = {}
        dev = self.device
        sd = {k: v.detach().to(torch.float32).cpu() for k, v in state_dict.items()}
        f8 = self._f8
        bf = lambda t: t.to(torch.bfloat16).contiguous().to(dev)               # noqa: E731
        f32 = lambda t: t.to(torch.float32).contiguous().to(dev)               # noqa: E731

        def lin(t, pt):
            return ops.quantize_mx(t.to(dev)) if f8(pt) else bf(t)

        def cnv(t, pt):
            if f8(pt):
                return ops.quantize_mx(t.permute(0, 2, 3, 1).reshape(t.shape[0], -1).contiguous().to(dev))
            return _pack_conv(t, torch).to(dev)
        D, g = spec.hidden, spec.grid
        # ---- BiT stem (bf16)
        p = "dpt.embeddings.backbone.bit."
        w = standardize(sd[p + "embedder.convolution.weight"])                  # [64, 3, 7, 7]
        kp = (49 * 3 + 63) // 64 * 64
        ws = torch.zeros(spec.stem, kp)
        ws[:, :147] = w.permute(0, 2, 3, 1).reshape(spec.stem, 147)
        self.w_stem, self.stem_kp = bf(ws), kp
        self.gn_stem = (f32(sd[p + "embedder.norm.weight"]), f32(sd[p + "embedder.norm.bias"]))
        self.bit = []
        for s, l, ci, mid, co, stride in spec.bit_layers():
            q = p + f"encoder.stages.{s}.layers.{l}."
            L = dict(stride=stride, mid=mid, co=co,
                     w1=bf(standardize(sd[q + "conv1.weight"]).reshape(mid, ci)),
                     w2=_pack_conv(standardize(sd[q + "conv2.weight"]), torch).to(dev),
                     w3=bf(standardize(sd[q + "conv3.weight"]).reshape(co, mid)))
            for n in ("1", "2", "3"):
                L["gn" + n] = (f32(sd[q + f"norm{n}.weight"]), f32(sd[q + f"norm{n}.bias"]))
            if l == 0:
                L["wd"] = bf(standardize(sd[q + "downsample.conv.weight"]).reshape(co, ci))
                L["gnd"] = (f32(sd[q + "downsample.norm.weight"]), f32(sd[q + "downsample.norm.bias"]))
            self.bit.append(L)
        # ---- embeddings (bf16 projection + position table)
        self.w_emb = bf(sd["dpt.embeddings.projection.weight"].reshape(D, spec.bit_widths[-1]))
        self.b_emb = f32(sd["dpt.embeddings.projection.bias"])
        pos = sd["dpt.embeddings.position_embeddings"][0]
        if pos.shape[0] != g * g + 1:
            raise ValueError("position table does not match the checkpoint grid")
        self.pos_tok, self.pos0 = f32(pos[1:]), f32(pos[0])
        self.cls = f32(sd["dpt.embeddings.cls_token"].reshape(D))
        # ---- encoder
        self.layers = []
        for i in range(spec.layers):
            q = f"dpt.encoder.layer.{i}."
            wq = torch.cat([sd[q + f"attention.attention.{n}.weight"] for n in ("query", "key", "value")], 0)
            bq = torch.cat([sd[q + f"attention.attention.{n}.bias"] for n in ("query", "key", "value")], 0)
            # softmax scale * log2(e) folded into the Q rows (fp32, before any rounding; see dpt.py)
            wq, bq = ops.fold_q_scale(wq, bq, 1.0 / math.sqrt(spec.hidden // spec.heads))
            self.layers.append(dict(
                ln1_g=f32(sd[q + "layernorm_before.weight"]), ln1_b=f32(sd[q + "layernorm_before.bias"]),
                w_qkv=lin(wq, "qkv"), b_qkv=f32(bq),
                w_o=lin(sd[q + "attention.output.dense.weight"], "o"), b_o=f32(sd[q + "attention.output.dense.bias"]),
                ln2_g=f32(sd[q + "layernorm_after.weight"]), ln2_b=f32(sd[q + "layernorm_after.bias"]),
                w_1=lin(sd[q + "intermediate.dense.weight"], "fc1"), b_1=f32(sd[q + "intermediate.dense.bias"]),
                w_2=lin(sd[q + "output.dense.weight"], "fc2"), b_2=f32(sd[q + "output.dense.bias"])))
        # ---- neck
        self.stages = []
        for i, (c, fac) in enumerate(zip(spec.neck, spec.factors)):
            st = dict(c=c, fac=fac, w_neck=cnv(sd[f"neck.convs.{i}.weight"], "neck"))
            if i >= 2:
                q = "neck.reassemble_stage."
                wr = sd[q + f"readout_projects.{i}.0.weight"]
                st.update(w_tok=lin(wr[:, :D], "readout"), w_cls=bf(wr[:, D:]),
                          b_ro=f32(sd[q + f"readout_projects.{i}.0.bias"]),
                          w_proj=lin(sd[q + f"layers.{i}.projection.weight"].reshape(c, D), "readout"),
                          b_proj=f32(sd[q + f"layers.{i}.projection.bias"]))
                if fac < 1:
                    st["w_rs"] = cnv(sd[q + f"layers.{i}.resize.weight"], "readout")
                    st["b_rs"] = f32(sd[q + f"layers.{i}.resize.bias"])
            self.stages.append(st)
        F = spec.fusion
        self.fusion = []
        for i in range(len(spec.neck)):
            q = f"neck.fusion_stage.layers.{i}."
            fl = dict(w_proj=bf(sd[q + "projection.weight"].reshape(F, F)), b_proj=f32(sd[q + "projection.bias"]))
            for r in ("residual_layer1", "residual_layer2"):
                for cv in ("convolution1", "convolution2"):
                    fl[f"{r}.{cv}.w"] = cnv(sd[q + f"{r}.{cv}.weight"], "fusion")
                    fl[f"{r}.{cv}.b"] = f32(sd[q + f"{r}.{cv}.bias"])
            self.fusion.append(fl)
        self.w_h0 = cnv(sd["head.head.0.weight"], "head")
        self.b_h0 = f32(sd["head.head.0.bias"])
        self.w_h2 = _pack_conv(sd["head.head.2.weight"], torch).to(dev)
        self.b_h2 = f32(sd["head.head.2.bias"])
        self.w_h4 = f32(sd["head.head.4.weight"].reshape(32))
        self.b_h4 = float(sd["head.head.4.bias"].reshape(()).item())

    def _f8(self, point: str) -> bool:
        """Whether quantisation point `point` (FP8_POINTS) runs on the MX fp8 engine."""
        return self.dtype == "fp8" and point not in self.bf16_points

    # ------------------------------------------------------------------ buffers
    def buffers(self, B: int) -> dict:
        import torch
        if B in self._bufs:
            return self._bufs[B]
        s, dev = self.spec, self.device
        D, g = s.hidden, s.grid
        T = g * g + 1
        M = B * T
        e = lambda shape, dt=torch.bfloat16: torch.empty(shape, dtype=dt, device=dev)   # noqa: E731
        b = dict(x=e((M, D), torch.float32), qkv=e((M, 3 * D)), att=e((M, D)), rb=e((B, D), torch.float32),
                 hs=[e((M, D)) for _ in range(2)], lnb=e((M, D)), mlpb=e((M, s.mlp)))
        if self.dtype == "fp8":
            b.update(ln=ops.empty_fp8((M, D), dev), att8=ops.empty_fp8((M, D), dev), mlp=ops.empty_fp8((M, s.mlp), dev),
                     tok8=[ops.empty_fp8((B * g * g, D), dev) for _ in range(2)])
        self._bufs[B] = b
        return b

    # ------------------------------------------------------------------ forward
    def forward(self, pixels, B: int, gh: int = None, gw: int = None):
        s = self.spec
        if tuple(pixels.shape[-2:]) != (s.image, s.image):
            raise ValueError(f"DPT-Hybrid runs on its {s.image}x{s.image} checkpoint grid, got {tuple(pixels.shape)}")
        feats_bit = self._bit(pixels, B)
        D, g = s.hidden, s.grid
        np_, T = g * g, g * g + 1
        buf = self.buffers(B)
        x = buf["x"]
        f3 = feats_bit[2]
        ops.linear(f3.view(B * np_, f3.shape[-1]), self.w_emb, bias=self.b_emb, table=self.pos_tok, table_rows=np_,
                   out=x, out_map=(np_, T, 1), rows=B * np_)
        ops.cls_pos(self.cls, self.pos0, x, B, T, D)
        scale = 1.0 / math.sqrt(D // s.heads)
        keep = list(s.out_indices[2:])
        f8 = self._f8
        for i, L in enumerate(self.layers):
            if f8("qkv"):
                ln = ops.layernorm_fp8(x, L["ln1_g"], L["ln1_b"], s.eps, out=buf["ln"])
                qkv = ops.linear_fp8(ln, L["w_qkv"], bias=L["b_qkv"], out=buf["qkv"])
            else:
                ln = ops.layernorm(x, L["ln1_g"], L["ln1_b"], s.eps, out=buf["lnb"])
                qkv = ops.linear(ln, L["w_qkv"], bias=L["b_qkv"], out=buf["qkv"])
            if f8("o"):       # the attention epilogue writes attention-out's fp8 operand directly
                att8 = ops.attention(qkv, B, T, s.heads, scale, out=buf["att8"], q_log2=True)
                ops.linear_fp8(att8, L["w_o"], bias=L["b_o"], res=x, out=x)
            else:
                att = ops.attention(qkv, B, T, s.heads, scale, out=buf["att"], q_log2=True)
                ops.linear(att, L["w_o"], bias=L["b_o"], res=x, out=x)
            if f8("fc1"):       # FC1's epilogue writes FC2's operand format
                ln = ops.layernorm_fp8(x, L["ln2_g"], L["ln2_b"], s.eps, out=buf["ln"])
                h = ops.linear_fp8(ln, L["w_1"], bias=L["b_1"], act="gelu",
                                   out=buf["mlp"] if f8("fc2") else buf["mlpb"], out_fp8=f8("fc2"))
            else:
                ln = ops.layernorm(x, L["ln2_g"], L["ln2_b"], s.eps, out=buf["lnb"])
                h = ops.linear(ln, L["w_1"], bias=L["b_1"], act="gelu", out=buf["mlpb"])
                if f8("fc2"):
                    h = ops.quant_fp8(h, out=buf["mlp"])
            if f8("fc2"):
                ops.linear_fp8(h, L["w_2"], bias=L["b_2"], res=x, out=x)
            else:
                ops.linear(h, L["w_2"], bias=L["b_2"], res=x, out=x)
            if i in keep:
                j = keep.index(i)
                ops.f32_to_bf16(x, out=buf["hs"][j])
                if f8("readout"):    # the readout's token rows (CLS skipped), quantised once
                    ops.quant_fp8(x, rows=B * np_, a_map=(np_, T, 1), out=buf["tok8"][j])
        feats = [self._neck_bit(0, feats_bit[0]), self._neck_bit(1, feats_bit[1])]
        feats += [self._reassemble_vit(j, buf, B) for j in (2, 3)]
        hidden = None
        for j, feat in enumerate(reversed(feats)):
            # the last stage's output feeds only the head: its upsample writes the head's fp8 operand
            hidden = self._fuse(self.fusion[j], feat, hidden, head_fp8=j == len(feats) - 1 and f8("head"))
        if f8("head"):
            t = ops.conv2d_fp8(hidden if isinstance(hidden, ops.Fp8) else ops.quant_fp8(hidden), self.w_h0, bias=self.b_h0)
        else:
            t = ops.conv2d(hidden, self.w_h0, bias=self.b_h0)
        return ops.head_upconv(t, 2 * t.shape[1], 2 * t.shape[2], self.w_h2, self.b_h2, self.w_h4, self.b_h4)

    __call__ = forward

    def _bit(self, pixels, B):
        """BiT-R50 stages 1-3 (bf16); returns the stage 1, 2, 3 maps (NHWC)."""
        s = self.spec
        cols, (oh, ow) = ops.stem_im2col(pixels.contiguous(), k_pitch=self.stem_kp)
        t = ops.linear(cols, self.w_stem).view(B, oh, ow, s.stem)
        t = ops.group_norm(t, *self.gn_stem, groups=s.groups, relu=True)
        x = ops.maxpool3s2(t)
        outs = []
        layers = s.bit_layers()
        for L, (st, l, ci, mid, co, stride) in zip(self.bit, layers):
            Bn, H, W, C = x.shape
            if stride == 2:
                OH, pt = ops.same_pad(H, 3, 2)
                OW, pl = ops.same_pad(W, 3, 2)
                short_in = ops.conv2d(x, L["wd"], k=1, stride=2, pad=0, out_hw=(OH, OW)) if l == 0 else None
            else:
                OH, OW, pt = H, W, 1
                short_in = ops.linear(x.view(-1, C), L["wd"]).view(Bn, H, W, co) if l == 0 else None
            y = ops.linear(x.view(-1, C), L["w1"]).view(Bn, H, W, mid)
            y = ops.group_norm(y, *L["gn1"], groups=s.groups, relu=True)
            y = ops.conv2d(y, L["w2"], k=3, stride=stride, pad=pt, out_hw=(OH, OW))
            y = ops.group_norm(y, *L["gn2"], groups=s.groups, relu=True)
            y = ops.linear(y.view(-1, mid), L["w3"]).view(Bn, OH, OW, co)
            shortcut = (short_in, *L["gnd"]) if l == 0 else x
            x = ops.group_norm(y, *L["gn3"], groups=s.groups, relu=True, shortcut=shortcut)
            if l == s.bit_depths[st] - 1:
                outs.append(x)
        return outs

    def _neck_bit(self, j, f):
        st = self.stages[j]
        if self._f8("neck"):
            return ops.conv2d_fp8(ops.quant_fp8(f), st["w_neck"])
        return ops.conv2d(f, st["w_neck"])

    def _reassemble_vit(self, j, buf, B):
        s, st = self.spec, self.stages[j]
        D, g = s.hidden, s.grid
        np_, T = g * g, g * g + 1
        k = j - 2
        hs = buf["hs"][k]
        rb = ops.linear(hs, st["w_cls"], bias=st["b_ro"], rows=B, a_map=(1, T, 0), out=buf["rb"])
        c = st["c"]
        f8n = self._f8("neck")
        if self._f8("readout"):
            # the last readout GEMM writes the neck conv's operand format
            sub = st["fac"] < 1
            tok = ops.linear_fp8(buf["tok8"][k], st["w_tok"], row_bias=rb, row_bias_group=np_, act="gelu", out_fp8=True)
            proj = ops.linear_fp8(tok, st["w_proj"], bias=st["b_proj"], out_fp8=f8n or sub)
            proj = proj.view(B, g, g, c)
            if sub:
                proj = ops.conv2d_fp8(proj, st["w_rs"], bias=st["b_rs"], k=3, stride=2, pad=1, out_fp8=f8n)
        else:
            tok = ops.linear(hs, st["w_tok"], rows=B * np_, a_map=(np_, T, 1), row_bias=rb, row_bias_group=np_,
                             act="gelu")
            proj = ops.linear(tok, st["w_proj"], bias=st["b_proj"]).view(B, g, g, c)
            if st["fac"] < 1:
                proj = ops.conv2d(proj, st["w_rs"], bias=st["b_rs"], k=3, stride=2, pad=1)
            if f8n:
                proj = ops.quant_fp8(proj)
        return ops.conv2d_fp8(proj, st["w_neck"]) if f8n else ops.conv2d(proj, st["w_neck"])

    def _fuse(self, fl, feat, hidden, head_fp8=False):
        if not self._f8("fusion"):
            return super()._fuse(fl, feat, hidden)
        if hidden is None:
            h = feat
        else:
            if tuple(hidden.shape) != tuple(feat.shape):
                raise ValueError(f"fusion shapes {tuple(hidden.shape)} vs {tuple(feat.shape)}")
            t = ops.conv2d_fp8(ops.quant_fp8(feat), fl["residual_layer1.convolution1.w"],
                               bias=fl["residual_layer1.convolution1.b"], relu_in=True, act="relu", out_fp8=True)
            h = ops.conv2d_fp8(t, fl["residual_layer1.convolution2.w"], bias=fl["residual_layer1.convolution2.b"],
                               res=feat, res2=hidden)
        t = ops.conv2d_fp8(ops.quant_fp8(h), fl["residual_layer2.convolution1.w"],
                           bias=fl["residual_layer2.convolution1.b"], relu_in=True, act="relu", out_fp8=True)
        h2 = ops.conv2d_fp8(t, fl["residual_layer2.convolution2.w"], bias=fl["residual_layer2.convolution2.b"], res=h)
        B, H, W, F = h2.shape
        p = ops.linear(h2.view(B * H * W, F), fl["w_proj"], bias=fl["b_proj"]).view(B, H, W, F)
        return ops.upsample2x(p, out_fp8=head_fp8 and F % 128 == 0)
