"""DPT depth network (ViT backbone + reassemble/fusion neck + depth head) on MI355X.

Weights are taken in the transformers `DPTForDepthEstimation` state-dict layout
(transformers 5.15 modeling_dpt.py), so a local safetensors export of
Intel/dpt-large loads unchanged; every block runs on a hand-written gfx950
kernel from libi2pc.so (ops.py), bf16 operands with fp32 accumulation and an
fp32 residual stream:

  embeddings   preprocess (patch rows) -> GEMM + bias + pos table, CLS row   modeling_dpt.py:185-235
  encoder x L  LN -> QKV GEMM -> fused attention -> O GEMM (+res, fp32)
               -> LN -> FC1 GEMM (+GELU) -> FC2 GEMM (+res)                  modeling_dpt.py:101-254
  reassemble   readout "project" = GEMM over tokens with the CLS half folded
               into a per-image bias, GELU; 1x1 projection; ConvT (k=s) as a
               GEMM with a pixel-shuffle store / identity / 3x3 s2 conv       modeling_dpt.py:257-387
  neck convs   3x3 implicit-GEMM convs                                        modeling_dpt.py:643-645
  fusion x 4   pre-activation residual units as conv GEMMs with ReLU-on-load,
               ReLU / bias / residual epilogues; 1x1 projection evaluated at
               low resolution BEFORE the align_corners=True 2x upsample (both
               are linear and the bilinear weights sum to one, so they commute;
               4x fewer FLOPs)                                                 modeling_dpt.py:390-509
  head         3x3 conv -> 2x upsample -> 3x3 conv + ReLU -> 1x1 conv + ReLU  modeling_dpt.py:679-716

The module preallocates every activation buffer per batch size, so a forward
issues only kernel launches (capturable into a HIP graph).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

# The head's tail runs as one kernel (ops.head_upconv); False selects the unfused
# resize -> conv -> head_out sequence (kept for parity tests).
FUSED_HEAD = True
# LayerNorm folded through the GEMMs (i2pc.h "LayerNorm fold"): the attention-out / FC2
# residual epilogues also write the bf16 residual and per-64-column (mean, M2) partials,
# ln_rowstats turns them into per-row (rstd, -rstd*mean), and QKV / FC1 run on gamma-scaled
# weights with the normalisation applied in their epilogue -- no separate LayerNorm pass
# (47 of the 48 in DPT-Large; layer 0's LN1 follows the embeddings).  False: LN kernels.
LN_FOLD = True
# With the fold: the residual stream between the encoder GEMMs is the shifted bf16 copy itself
# (i2pc.h "bf16 residual stream": attention-out / FC2 read it as res + res_shift and write it back
# as bf16(x - ln_shift)), as in the torch-bf16 forward, instead of an fp32 stream plus a bf16 copy:
# those two epilogues move 76 MB instead of 189 MB per call at C2.  False: the fp32 stream.
BF16_STREAM = __import__("os").environ.get("I2PC_BF16_STREAM", "1") != "0"

from . import ops


@dataclass(frozen=True)
class DPTSpec:
    name: str
    hidden: int
    layers: int
    heads: int
    mlp: int
    patch: int
    image: int
    out_indices: tuple
    neck: tuple
    fusion: int
    factors: tuple = (4, 2, 1, 0.5)
    eps: float = 1e-12
    family: str = "dpt"

    @property
    def grid(self) -> int:
        return self.image // self.patch

    def hf_config_kwargs(self) -> dict:
        return dict(hidden_size=self.hidden, num_hidden_layers=self.layers, num_attention_heads=self.heads,
                    intermediate_size=self.mlp, patch_size=self.patch, image_size=self.image,
                    backbone_out_indices=list(self.out_indices), neck_hidden_sizes=list(self.neck),
                    fusion_hidden_size=self.fusion, reassemble_factors=list(self.factors),
                    layer_norm_eps=self.eps, readout_type="project", qkv_bias=True, hidden_act="gelu",
                    is_hybrid=False, add_projection=False, head_in_index=-1)

    def flops_per_image(self) -> float:
        """Algorithmic FLOPs (2 x MAC of every GEMM/conv + 4*T^2*d*L attention) as this module computes them."""
        g, D, T = self.grid, self.hidden, self.grid ** 2 + 1
        f = 2.0 * g * g * 3 * self.patch ** 2 * D                       # patch embed
        f += self.layers * 2.0 * T * (4 * D * D + 2 * D * self.mlp)      # QKV, O, FC1, FC2
        f += self.layers * 4.0 * T * T * D                              # attention
        F = self.fusion
        sizes = []
        for c, fac in zip(self.neck, self.factors):
            f += 2.0 * g * g * D * D + 2.0 * D * D                         # readout (tokens + CLS bias)
            f += 2.0 * g * g * D * c                                       # 1x1 projection
            if fac > 1:
                f += 2.0 * g * g * c * c * fac * fac
                s = int(g * fac)
            elif fac == 1:
                s = g
            else:
                s = (g + 1) // 2
                f += 2.0 * s * s * 9 * c * c
            f += 2.0 * s * s * 9 * c * F                                   # neck conv
            sizes.append(s)
        for j, s in enumerate(reversed(sizes)):
            units = 1 if j == 0 else 2
            f += units * 2 * 2.0 * s * s * 9 * F * F                       # residual units
            f += 2.0 * s * s * F * F                                       # projection at low res
        s = 2 * sizes[0]
        f += 2.0 * s * s * 9 * F * (F // 2)
        f += 2.0 * (2 * s) ** 2 * 9 * (F // 2) * 32 + 2.0 * (2 * s) ** 2 * 32
        return f


DPT_LARGE = DPTSpec("dpt-large", hidden=1024, layers=24, heads=16, mlp=4096, patch=16, image=384,
                    out_indices=(5, 11, 17, 23), neck=(256, 512, 1024, 1024), fusion=256)
# a small member of the same family for fast parity tests
DPT_TINY = DPTSpec("dpt-tiny", hidden=128, layers=4, heads=2, mlp=256, patch=16, image=128,
                   out_indices=(0, 1, 2, 3), neck=(64, 128, 256, 256), fusion=128)


def state_dict_keys(spec: DPTSpec) -> dict:
    """name -> shape of every tensor DPTForDepthEstimation(config) holds (transformers key layout)."""
    D, P, T = spec.hidden, spec.patch, spec.grid ** 2 + 1
    k = {
        "dpt.embeddings.cls_token": (1, 1, D),
        "dpt.embeddings.position_embeddings": (1, T, D),
        "dpt.embeddings.patch_embeddings.projection.weight": (D, 3, P, P),
        "dpt.embeddings.patch_embeddings.projection.bias": (D,),
        "dpt.layernorm.weight": (D,), "dpt.layernorm.bias": (D,),
    }
    for i in range(spec.layers):
        p = f"dpt.encoder.layer.{i}."
        for n in ("query", "key", "value"):
            k[p + f"attention.attention.{n}.weight"] = (D, D)
            k[p + f"attention.attention.{n}.bias"] = (D,)
        k[p + "attention.output.dense.weight"] = (D, D)
        k[p + "attention.output.dense.bias"] = (D,)
        k[p + "intermediate.dense.weight"] = (spec.mlp, D)
        k[p + "intermediate.dense.bias"] = (spec.mlp,)
        k[p + "output.dense.weight"] = (D, spec.mlp)
        k[p + "output.dense.bias"] = (D,)
        for n in ("layernorm_before", "layernorm_after"):
            k[p + n + ".weight"] = (D,)
            k[p + n + ".bias"] = (D,)
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
        k[f"neck.reassemble_stage.readout_projects.{i}.0.weight"] = (D, 2 * D)
        k[f"neck.reassemble_stage.readout_projects.{i}.0.bias"] = (D,)
        k[f"neck.convs.{i}.weight"] = (F, c, 3, 3)
        p = f"neck.fusion_stage.layers.{i}."
        k[p + "projection.weight"] = (F, F, 1, 1)
        k[p + "projection.bias"] = (F,)
        for r in ("residual_layer1", "residual_layer2"):
            for cv in ("convolution1", "convolution2"):
                k[p + f"{r}.{cv}.weight"] = (F, F, 3, 3)
                k[p + f"{r}.{cv}.bias"] = (F,)
    k["head.head.0.weight"] = (F // 2, F, 3, 3)
    k["head.head.0.bias"] = (F // 2,)
    k["head.head.2.weight"] = (32, F // 2, 3, 3)
    k["head.head.2.bias"] = (32,)
    k["head.head.4.weight"] = (1, 32, 1, 1)
    k["head.head.4.bias"] = (1,)
    return k


def synthetic_state_dict(spec: DPTSpec, seed: int = 0):
    """Deterministic random weights (no pretrained checkpoint is available offline).

    Fan-in-scaled normal weights keep activations O(1) through the network and a
    positive final bias keeps the ReLU depth non-trivial; speed is weight-independent.
    """
    import torch
    g = torch.Generator(device="cpu").manual_seed(seed)
    sd = {}
    for name, shape in state_dict_keys(spec).items():
        if name.endswith("cls_token"):
            t = 0.5 * torch.randn(shape, generator=g)
        elif name.endswith("position_embeddings"):
            t = 0.1 * torch.randn(shape, generator=g)
        elif "layernorm" in name and name.endswith("weight"):
            t = 1.0 + 0.1 * torch.randn(shape, generator=g)
        elif name == "head.head.4.bias":
            t = torch.full(shape, 2.0)
        elif name.endswith("bias"):
            t = 0.02 * torch.randn(shape, generator=g)
        elif name == "head.head.4.weight":
            t = 0.5 * torch.randn(shape, generator=g) / math.sqrt(32)
        elif name.endswith("resize.weight") and len(shape) == 4 and shape[2] == shape[3] and shape[2] in (2, 4) \
                and "reassemble" in name:
            t = torch.randn(shape, generator=g) / math.sqrt(shape[0])
        else:
            fan_in = int(torch.tensor(shape[1:]).prod())
            t = torch.randn(shape, generator=g) / math.sqrt(fan_in)
        sd[name] = t.float()
    return sd


def _pack_conv(w, torch):
    """[Co, Ci, k, k] -> bf16 [Co, k*k*Ci] with (ky, kx, ci) order (NHWC implicit GEMM)."""
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1).to(torch.bfloat16).contiguous()


@dataclass
class _Buffers:
    B: int
    t: dict = field(default_factory=dict)


class DPTDepthModel:
    """bf16 DPT forward on MI355X.  `forward(patches, B)` -> depth fp32 [B, image, image]."""

    def __init__(self, spec: DPTSpec, state_dict: dict, device):
        import torch
        self.spec = spec
        self.device = torch.device(device)
        self._bufs = {}
        dev = self.device
        sd = {k: v.detach().to(torch.float32).cpu() for k, v in state_dict.items()}
        bf = lambda t: t.to(torch.bfloat16).contiguous().to(dev)     # noqa: E731
        f32 = lambda t: t.to(torch.float32).contiguous().to(dev)     # noqa: E731
        D, P, g = spec.hidden, spec.patch, spec.grid
        pe = sd["dpt.embeddings.patch_embeddings.projection.weight"]
        self.w_pe = bf(pe.reshape(D, 3 * P * P))
        self.b_pe = f32(sd["dpt.embeddings.patch_embeddings.projection.bias"])
        pos = sd["dpt.embeddings.position_embeddings"][0]
        g0 = int(round(math.sqrt(pos.shape[0] - 1)))
        if g0 * g0 != pos.shape[0] - 1:
            raise ValueError(f"position table of {pos.shape[0]} rows is not a square grid + CLS")
        self._pos_grid = f32(pos[1:]).view(g0, g0, D)
        self._pos_tables = {}
        self.pos_tok = self._pos_table(g, g)
        self.pos0 = f32(pos[0])
        self.cls = f32(sd["dpt.embeddings.cls_token"].reshape(D))
        self.layers = []
        for i in range(spec.layers):
            p = f"dpt.encoder.layer.{i}."
            q = [sd[p + f"attention.attention.{n}.weight"] for n in ("query", "key", "value")]
            qb = [sd[p + f"attention.attention.{n}.bias"] for n in ("query", "key", "value")]
            # softmax scale * log2(e) folded into the Q rows (fp32, before the bf16 rounding): the QKV GEMM
            # writes Q in the exp2 domain that attention(..., q_log2=True) takes
            wq, bq = ops.fold_q_scale(torch.cat(q, 0), torch.cat(qb, 0), 1.0 / math.sqrt(spec.hidden // spec.heads))
            q, qb = [wq], [bq]
            L = dict(
                ln1_g=f32(sd[p + "layernorm_before.weight"]), ln1_b=f32(sd[p + "layernorm_before.bias"]),
                w_qkv=bf(torch.cat(q, 0)), b_qkv=f32(torch.cat(qb, 0)),
                w_o=bf(sd[p + "attention.output.dense.weight"]), b_o=f32(sd[p + "attention.output.dense.bias"]),
                ln2_g=f32(sd[p + "layernorm_after.weight"]), ln2_b=f32(sd[p + "layernorm_after.bias"]),
                w_1=bf(sd[p + "intermediate.dense.weight"]), b_1=f32(sd[p + "intermediate.dense.bias"]),
                w_2=bf(sd[p + "output.dense.weight"]), b_2=f32(sd[p + "output.dense.bias"]),
            )
            # the LN-folded forms: W' = bf16(W * gamma), col_sum = sum_k W', bias' = b + W beta
            wf, cs, bfold = ops.ln_fold_weights(torch.cat(q, 0), torch.cat(qb, 0), sd[p + "layernorm_before.weight"],
                                                sd[p + "layernorm_before.bias"])
            L.update(w_qkv_f=wf.to(dev), s_qkv=cs.to(dev), b_qkv_f=bfold.to(dev))
            wf, cs, bfold = ops.ln_fold_weights(sd[p + "intermediate.dense.weight"], sd[p + "intermediate.dense.bias"],
                                                sd[p + "layernorm_after.weight"], sd[p + "layernorm_after.bias"])
            L.update(w_1_f=wf.to(dev), s_1=cs.to(dev), b_1_f=bfold.to(dev))
            self.layers.append(L)
        self.stages = []
        for i, (c, fac) in enumerate(zip(spec.neck, spec.factors)):
            p = f"neck.reassemble_stage."
            wr = sd[p + f"readout_projects.{i}.0.weight"]
            st = dict(c=c, fac=fac,
                      w_tok=bf(wr[:, :D]), w_cls=bf(wr[:, D:]), b_ro=f32(sd[p + f"readout_projects.{i}.0.bias"]),
                      w_proj=bf(sd[p + f"layers.{i}.projection.weight"].reshape(c, D)),
                      b_proj=f32(sd[p + f"layers.{i}.projection.bias"]),
                      w_neck=_pack_conv(sd[f"neck.convs.{i}.weight"], torch).to(dev))
            if fac > 1:
                s = int(fac)
                w = sd[p + f"layers.{i}.resize.weight"]                     # [Ci, Co, s, s]
                st["w_rs"] = bf(w.permute(2, 3, 1, 0).reshape(s * s * c, c))
                st["b_rs"] = f32(sd[p + f"layers.{i}.resize.bias"].repeat(s * s))
            elif fac < 1:
                st["w_rs"] = _pack_conv(sd[p + f"layers.{i}.resize.weight"], torch).to(dev)
                st["b_rs"] = f32(sd[p + f"layers.{i}.resize.bias"])
            self.stages.append(st)
        F = spec.fusion
        self.fusion = []
        for i in range(len(spec.neck)):
            p = f"neck.fusion_stage.layers.{i}."
            fl = dict(w_proj=bf(sd[p + "projection.weight"].reshape(F, F)), b_proj=f32(sd[p + "projection.bias"]))
            for r in ("residual_layer1", "residual_layer2"):
                for cv in ("convolution1", "convolution2"):
                    fl[f"{r}.{cv}.w"] = _pack_conv(sd[p + f"{r}.{cv}.weight"], torch).to(dev)
                    fl[f"{r}.{cv}.b"] = f32(sd[p + f"{r}.{cv}.bias"])
            self.fusion.append(fl)
        self.w_h0 = _pack_conv(sd["head.head.0.weight"], torch).to(dev)
        self.b_h0 = f32(sd["head.head.0.bias"])
        self.w_h2 = _pack_conv(sd["head.head.2.weight"], torch).to(dev)
        self.b_h2 = f32(sd["head.head.2.bias"])
        self.w_h4 = f32(sd["head.head.4.weight"].reshape(32))
        self.b_h4 = float(sd["head.head.4.bias"].reshape(()).item())

    def _pos_table(self, gh: int, gw: int):
        """Position rows for a gh x gw patch grid: DPTViTEmbeddings._resize_pos_embed
        (modeling_dpt.py:202-214, bilinear, align_corners=False).  A one-time parameter
        transform per grid size, done with torch on the device and cached."""
        key = (gh, gw)
        if key not in self._pos_tables:
            import torch
            g0 = self._pos_grid.shape[0]
            if (gh, gw) == (g0, g0):
                t = self._pos_grid.reshape(g0 * g0, -1).contiguous()
            else:
                grid = self._pos_grid.permute(2, 0, 1).unsqueeze(0)
                t = torch.nn.functional.interpolate(grid, size=(gh, gw), mode="bilinear")
                t = t[0].permute(1, 2, 0).reshape(gh * gw, -1).contiguous()
            self._pos_tables[key] = t
        return self._pos_tables[key]

    # ------------------------------------------------------------------ buffers
    def buffers(self, B: int, gh: int = None, gw: int = None) -> dict:
        import torch
        s, dev = self.spec, self.device
        gh, gw = gh or s.grid, gw or s.grid
        if (B, gh, gw) in self._bufs:
            return self._bufs[(B, gh, gw)]
        D = s.hidden
        T = gh * gw + 1
        M = B * T
        e = lambda shape, dt=torch.bfloat16: torch.empty(shape, dtype=dt, device=dev)   # noqa: E731
        b = dict(x=e((M, D), torch.float32), ln=e((M, D)), qkv=e((M, 3 * D)), att=e((M, D)), mlp=e((M, s.mlp)),
                 hs=[e((M, D)) for _ in s.out_indices], rb=e((B, D), torch.float32), tok=e((B * gh * gw, D)),
                 part=e((M, D // 64, 2), torch.float32), rs=e((M, 2), torch.float32), shift=e((M,), torch.float32),
                 shift2=e((M,), torch.float32))
        b["ln_fold"] = LN_FOLD and D % 64 == 0 and self._ln_fold_ok(b, M)
        self._bufs[(B, gh, gw)] = b
        return b

    def _ln_fold_ok(self, b, M) -> bool:
        """Whether libi2pc.so runs the LN-folded calls at this batch (asked of the C side:
        i2pc_gemm_kernel_name is "invalid" for a descriptor i2pc_gemm would reject)."""
        s, L = self.spec, self.layers[0]
        D = s.hidden

        def name(x, w, out, **kw):
            d = ops.GemmDesc()
            d.a, d.lda, d.m, d.n, d.k = x.data_ptr(), x.stride(0), M, w.shape[0], w.shape[1]
            d.w, d.ldw, d.c, d.ldc = w.data_ptr(), w.stride(0), out.data_ptr(), out.stride(0)
            d.c_f32 = int(out.dtype.is_floating_point and out.element_size() == 4)
            for k, v in kw.items():
                setattr(d, k, v)
            return ops.gemm_kernel_label(d)
        consumer = dict(ln_rows=b["rs"].data_ptr(), col_sum=L["s_qkv"].data_ptr(), bias=L["b_qkv_f"].data_ptr())
        producer = dict(res=b["x"].data_ptr(), res_f32=1, ldr=D, ln_part=b["part"].data_ptr(),
                        c_bf16=b["ln"].data_ptr(), ldc_bf16=D, ln_shift=b["shift"].data_ptr())
        names = [name(b["ln"], L["w_qkv_f"], b["qkv"], **consumer),
                 name(b["ln"], L["w_1_f"], b["mlp"], **dict(consumer, col_sum=L["s_1"].data_ptr(), act=1)),
                 name(b["att"], L["w_o"], b["x"], **producer),
                 name(b["mlp"], L["w_2"], b["x"], **producer)]
        if BF16_STREAM:   # bf16-output producers (layer 0's attention-out still reads the fp32 embeddings)
            stream = dict(res=b["ln"].data_ptr(), res_f32=0, ldr=D, ln_part=b["part"].data_ptr(),
                          ln_shift=b["shift"].data_ptr(), res_shift=b["shift2"].data_ptr())
            names += [name(b["att"], L["w_o"], b["ln"], **dict(producer, c_bf16=0, ldc_bf16=0)),
                      name(b["att"], L["w_o"], b["ln"], **stream),
                      name(b["mlp"], L["w_2"], b["ln"], **stream)]
        return "invalid" not in names

    # ------------------------------------------------------------------ forward
    def forward(self, patches, B: int, gh: int = None, gw: int = None):
        """patches: bf16 [B * gh * gw, 3*patch^2] (preprocess layout 'patches') -> depth fp32 [B, H', W'].
        Any patch grid (the position table is interpolated as DPTViTEmbeddings does); the Intel
        processors resize to the square checkpoint grid."""
        s = self.spec
        gh, gw = gh or s.grid, gw or s.grid
        D = s.hidden
        np_, T = gh * gw, gh * gw + 1
        self._grid = (gh, gw)
        buf = self.buffers(B, gh, gw)
        x = buf["x"]
        # embeddings: patch GEMM + bias + position table written into token rows 1..T-1; CLS row
        ops.linear(patches, self.w_pe, bias=self.b_pe, table=self._pos_table(gh, gw), table_rows=np_, out=x,
                   out_map=(np_, T, 1), rows=B * np_)
        ops.cls_pos(self.cls, self.pos0, x, B, T, D)
        scale = 1.0 / math.sqrt(D // s.heads)
        hs_i = 0
        fold = buf["ln_fold"]
        a_in = None          # LN fold: the bf16 residual rows the previous FC2 wrote (rows scaled by buf["rs"])
        nl = len(self.layers)
        for i, L in enumerate(self.layers):
            if not fold:
                ln = ops.layernorm(x, L["ln1_g"], L["ln1_b"], s.eps, out=buf["ln"])
                qkv = ops.linear(ln, L["w_qkv"], bias=L["b_qkv"], out=buf["qkv"])
                att = ops.attention(qkv, B, T, s.heads, scale, out=buf["att"], q_log2=True)
                ops.linear(att, L["w_o"], bias=L["b_o"], res=x, out=x)
                ln = ops.layernorm(x, L["ln2_g"], L["ln2_b"], s.eps, out=buf["ln"])
                h = ops.linear(ln, L["w_1"], bias=L["b_1"], act="gelu", out=buf["mlp"])
                ops.linear(h, L["w_2"], bias=L["b_2"], res=x, out=x)
                if i in s.out_indices:
                    ops.f32_to_bf16(x, out=buf["hs"][hs_i])
                    hs_i += 1
                continue
            if a_in is None:      # layer 0: LN1 of the embeddings (its row means: the first shift)
                ln = ops.layernorm(x, L["ln1_g"], L["ln1_b"], s.eps, out=buf["ln"], mean_out=buf["shift"])
                qkv = ops.linear(ln, L["w_qkv"], bias=L["b_qkv"], out=buf["qkv"])
            else:
                qkv = ops.linear(a_in, L["w_qkv_f"], bias=L["b_qkv_f"], ln_rows=buf["rs"], col_sum=L["s_qkv"],
                                 out=buf["qkv"])
            att = ops.attention(qkv, B, T, s.heads, scale, out=buf["att"], q_log2=True)
            if BF16_STREAM:
                a_in = self._stream_layer(i, L, att, a_in, buf)
                continue
            # the residual's bf16 copy is stored minus the previous LayerNorm's row mean (shift),
            # so rows whose mean is large against their spread keep their precision
            ops.linear(att, L["w_o"], bias=L["b_o"], res=x, out=x, ln_part=buf["part"], out_bf16=buf["ln"],
                       ln_shift=buf["shift"])
            ops.ln_rowstats(buf["part"], s.eps, out=buf["rs"], shift_in=buf["shift"], shift_out=buf["shift"])
            h = ops.linear(buf["ln"], L["w_1_f"], bias=L["b_1_f"], act="gelu", ln_rows=buf["rs"], col_sum=L["s_1"],
                           out=buf["mlp"])
            # FC2 + residual; its bf16 copy is the next QKV's A -- shifted like the one above, except
            # for a kept hidden state, which the neck reads as it is (unshifted)
            if i in s.out_indices:
                dst, shift = buf["hs"][hs_i], None
                hs_i += 1
            else:
                dst, shift = buf["ln"], buf["shift"]
            ops.linear(h, L["w_2"], bias=L["b_2"], res=x, out=x, ln_part=buf["part"], out_bf16=dst, ln_shift=shift)
            if i + 1 < nl:
                ops.ln_rowstats(buf["part"], s.eps, out=buf["rs"], shift_in=shift, shift_out=buf["shift"])
            a_in = dst
        feats = [self._reassemble(j, buf["hs"][j], B, buf) for j in range(len(self.stages))]
        hidden = None
        for j, feat in enumerate(reversed(feats)):
            hidden = self._fuse(self.fusion[j], feat, hidden)
        t = ops.conv2d(hidden, self.w_h0, bias=self.b_h0)
        if FUSED_HEAD:       # 2x upsample + 3x3 conv + ReLU + 1x1 conv + ReLU in one kernel
            return ops.head_upconv(t, 2 * t.shape[1], 2 * t.shape[2], self.w_h2, self.b_h2, self.w_h4, self.b_h4)
        u = ops.upsample2x(t)
        t2 = ops.conv2d(u, self.w_h2, bias=self.b_h2, act="relu")
        return ops.head_out(t2, self.w_h4, self.b_h4)

    __call__ = forward

    def _stream_layer(self, i, L, att, a_in, buf):
        """The rest of encoder layer i on the shifted bf16 residual stream (BF16_STREAM): attention-out
        and FC2 read the stream (a_in, stored relative to the shift buf["_rsh"]; layer 0: the fp32
        embeddings) and write it back relative to the latest LayerNorm mean; ln_rowstats alternates
        between the two shift buffers (the one the stream is stored relative to is never overwritten
        while it is read).  Layers whose hidden state the neck reads store it unshifted (shift 0).
        Returns the stream after FC2 (the next QKV's A)."""
        s = self.spec
        kept = i in s.out_indices
        sh = (buf["shift"], buf["shift2"])
        if a_in is None:          # layer 0: the residual is the fp32 embeddings; LN1's means are in shift
            res, rsh, cur = buf["x"], None, 0
        else:
            res, rsh, cur = a_in, buf["_rsh"], buf["_cur"]
        # attention-out: stream -> buf["ln"], relative to sh[cur] (LN1's mean)
        ops.linear(att, L["w_o"], bias=L["b_o"], res=res, res_shift=rsh, out=buf["ln"], ln_part=buf["part"],
                   ln_shift=sh[cur])
        ops.ln_rowstats(buf["part"], s.eps, out=buf["rs"], shift_in=sh[cur], shift_out=sh[cur ^ 1])
        h = ops.linear(buf["ln"], L["w_1_f"], bias=L["b_1_f"], act="gelu", ln_rows=buf["rs"], col_sum=L["s_1"],
                       out=buf["mlp"])
        # FC2: stream -> buf["ln"] in place relative to sh[cur ^ 1] (LN2's mean), or a kept hidden state
        if kept:
            dst, osh = buf["hs"][s.out_indices.index(i)], None
        else:
            dst, osh = buf["ln"], sh[cur ^ 1]
        ops.linear(h, L["w_2"], bias=L["b_2"], res=buf["ln"], res_shift=sh[cur], out=dst, ln_part=buf["part"],
                   ln_shift=osh)
        if i + 1 < len(self.layers):
            ops.ln_rowstats(buf["part"], s.eps, out=buf["rs"], shift_in=osh, shift_out=sh[cur])
        buf["_rsh"], buf["_cur"] = osh, cur
        return dst

    def _reassemble(self, j, hs, B, buf):
        s, st = self.spec, self.stages[j]
        D = s.hidden
        gh, gw = getattr(self, "_grid", (s.grid, s.grid))
        np_, T = gh * gw, gh * gw + 1
        rb = ops.linear(hs, st["w_cls"], bias=st["b_ro"], rows=B, a_map=(1, T, 0), out=buf["rb"])
        tok = ops.linear(hs, st["w_tok"], rows=B * np_, a_map=(np_, T, 1), row_bias=rb, row_bias_group=np_,
                         act="gelu", out=buf["tok"])
        c = st["c"]
        proj = ops.linear(tok, st["w_proj"], bias=st["b_proj"]).view(B, gh, gw, c)
        fac = st["fac"]
        if fac > 1:
            r = ops.conv_transpose(proj, st["w_rs"], st["b_rs"], int(fac))
        elif fac == 1:
            r = proj
        else:
            r = ops.conv2d(proj, st["w_rs"], bias=st["b_rs"], k=3, stride=2, pad=1)
        return ops.conv2d(r, st["w_neck"])

    def _fuse(self, fl, feat, hidden):
        if hidden is None:
            h = feat
        else:
            if tuple(hidden.shape) != tuple(feat.shape):   # odd grids: modeling_dpt.py:696-699
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
        return ops.upsample2x(p)
