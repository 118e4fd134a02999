"""Llama-3 (+LoRA) for sequence classification on packed batches (BASELINE.json config 5).

Not in the reference; required by the north star ("Llama-3-8B LoRA 8-client serverless async
P2P, delta-only exchange, 288 GB HBM sizing"). Base weights are frozen bf16 and live OUTSIDE the
federated flat buffer; only LoRA adapters on q,k,v,o,gate,up,down plus the score head are
trainable and exchanged (~42 M params at r=16 for 8B = 84 MB bf16 per exchange).

MI355X layout: q|k|v projections fused into one [(nh+2nkv)*d, H] weight, gate|up fused into one
[2I, H] weight (one GEMM each); RoPE rotates the q,k column blocks of the packed projection in
place; attention is causal GQA varlen flash attention (d=128).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from .. import ops
from ..data.batching import PackedBatch
from ..ops import ref
from .common import SeqClassifierBase, new_param, row_slice, whole


@dataclass
class LlamaConfig:
    vocab_size: int = 128256
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 8
    max_position_embeddings: int = 8192
    rms_norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    num_labels: int = 2
    initializer_range: float = 0.02
    lora_rank: int = 16
    lora_alpha: float = 32.0
    lora_targets: tuple = ("q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj")
    cls_token_id: int = 128000
    sep_token_id: int = 128001
    pad_token_id: int = 128004

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads


class LoRA(nn.Module):
    """Low-rank adapters for a fused projection: one (A_i, B_i) pair per output block."""

    def __init__(self, in_features: int, out_blocks: List[int], r: int, alpha: float, device, dtype):
        super().__init__()
        self.r, self.scale = r, alpha / r
        self.out_blocks = out_blocks
        bound = 1.0 / math.sqrt(in_features)  # kaiming_uniform(a=sqrt(5)) bound
        A = torch.empty(len(out_blocks) * r, in_features, device=device, dtype=dtype).uniform_(-bound, bound)
        self.A = nn.Parameter(A)                               # [n*r, in] (A_i stacked)
        self.B = nn.ParameterList([new_param((o, r), device, dtype, "zeros") for o in out_blocks])

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        xa = ops.linear(x, self.A)  # [T, n*r]: ONE GEMM for all blocks
        outs = [ops.linear(xa[:, i * self.r:(i + 1) * self.r], B) for i, B in enumerate(self.B)]
        d = outs[0] if len(outs) == 1 else torch.cat(outs, dim=1)
        return d * self.scale

    def fused(self, x: torch.Tensor, w: torch.Tensor,
              residual: Optional[torch.Tensor] = None) -> torch.Tensor:
        """x W^T + this adapter's delta (+ ``residual``), WITHOUT materialising the delta or the
        sum as separate passes: the low-rank product is a tail of the base GEMM's reduction and
        the residual add its epilogue (ops.lora_linear; GPU). CPU: the unfused reference."""
        return ops.lora_linear(x, w, self.A, list(self.B), self.scale, residual)


class LlamaLayer(nn.Module):
    def __init__(self, cfg: LlamaConfig, device, dtype, lora: bool):
        super().__init__()
        H, I, d = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
        nh, nkv, std = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.initializer_range
        self.cfg = cfg
        rg = not lora
        self.in_ln = new_param((H,), device, dtype, "ones", requires_grad=rg)
        self.post_ln = new_param((H,), device, dtype, "ones", requires_grad=rg)
        self.qkv_weight = new_param(((nh + 2 * nkv) * d, H), device, dtype, "normal", std, rg)
        self.o_weight = new_param((H, nh * d), device, dtype, "normal", std, rg)
        self.gate_up_weight = new_param((2 * I, H), device, dtype, "normal", std, rg)
        self.down_weight = new_param((H, I), device, dtype, "normal", std, rg)
        self.lora = lora
        if lora:
            r, a = cfg.lora_rank, cfg.lora_alpha
            self.lora_qkv = LoRA(H, [nh * d, nkv * d, nkv * d], r, a, device, dtype)
            self.lora_o = LoRA(nh * d, [H], r, a, device, dtype)
            self.lora_gate_up = LoRA(H, [I, I], r, a, device, dtype)
            self.lora_down = LoRA(I, [H], r, a, device, dtype)

    def forward(self, x, batch: PackedBatch, cos, sin, rows=None):
        c = self.cfg
        nh, nkv, d = c.num_attention_heads, c.num_key_value_heads, c.head_dim
        h = ops.rmsnorm(x, self.in_ln, c.rms_norm_eps)
        qkv = self.lora_qkv.fused(h, self.qkv_weight) if self.lora else ops.linear(h, self.qkv_weight)
        qkv = ops.rope(qkv, batch.position_ids, cos, sin, nh, nkv, d)
        if rows is None:
            ctx = ops.varlen_attention(qkv, batch.cu_seqlens, batch.cu_host, batch.max_seqlen,
                                       nh, nkv, d, 0.0, self.training, causal=True,
                                       sched=getattr(batch, "attn_sched", None))
        else:  # last layer: only the pooled last-token rows are consumed
            ctx = ops.query_subset_attention(qkv, rows, batch.cu_seqlens, batch.max_seqlen, nh,
                                             nkv, d, 0.0, self.training, causal=True)
            x = x.index_select(0, rows.long())
        if self.lora:   # residual adds fused into the projections' GEMM epilogues
            x = self.lora_o.fused(ctx, self.o_weight, residual=x)
        else:
            x = x + ops.linear(ctx, self.o_weight)
        h2 = ops.rmsnorm(x, self.post_ln, c.rms_norm_eps)
        if self.lora:   # SwiGLU and the residual add in the projections' GEMM epilogues
            gl, dl = self.lora_gate_up, self.lora_down
            return ops.lora_swiglu_mlp(h2, self.gate_up_weight, gl.A, list(gl.B), gl.scale,
                                       self.down_weight, dl.A, list(dl.B), dl.scale, x)
        a = ops.swiglu(ops.linear(h2, self.gate_up_weight))
        return x + ops.linear(a, self.down_weight)


class LlamaForSequenceClassification(SeqClassifierBase):
    hf_architecture = "LlamaForSequenceClassification"
    hf_model_type = "llama"

    def __init__(self, cfg: LlamaConfig, device=None, dtype=torch.bfloat16, lora: bool = True):
        super().__init__()
        H = cfg.hidden_size
        self.cfg, self.lora = cfg, lora
        rg = not lora
        self.embed_tokens = new_param((cfg.vocab_size, H), device, dtype, "normal",
                                      cfg.initializer_range, rg)
        self.layers = nn.ModuleList([LlamaLayer(cfg, device, dtype, lora)
                                     for _ in range(cfg.num_hidden_layers)])
        self.norm = new_param((H,), device, dtype, "ones", requires_grad=rg)
        self.score_weight = new_param((cfg.num_labels, H), device, dtype, "normal", cfg.initializer_range)
        cos, sin = ref.rope_cache(cfg.max_position_embeddings, cfg.head_dim, cfg.rope_theta, device)
        self.register_buffer("rope_cos", cos, persistent=False)
        self.register_buffer("rope_sin", sin, persistent=False)

    def forward(self, batch: PackedBatch, token_type_ids=None):
        x = torch.nn.functional.embedding(batch.input_ids.long(), self.embed_tokens)
        rows = batch.cu_seqlens[1:batch.n_seq + 1] - 1
        n = len(self.layers) - 1
        for i, layer in enumerate(self.layers):
            x = layer(x, batch, self.rope_cos, self.rope_sin,
                      rows if (i == n and self.pooled_rows_only) else None)
        last = x if self.pooled_rows_only else x.index_select(0, rows.long())
        last = ops.rmsnorm(last, self.norm, self.cfg.rms_norm_eps)
        return ops.linear(last, self.score_weight)

    # HF names ---------------------------------------------------------------------------
    def hf_items(self):
        c = self.cfg
        d, nh, nkv, I = c.head_dim, c.num_attention_heads, c.num_key_value_heads, c.intermediate_size
        it = [("model.embed_tokens.weight", *whole(self.embed_tokens))]
        for i, L in enumerate(self.layers):
            p = f"model.layers.{i}."
            it += [
                (p + "self_attn.q_proj.weight", *row_slice(L.qkv_weight, 0, nh * d)),
                (p + "self_attn.k_proj.weight", *row_slice(L.qkv_weight, nh * d, (nh + nkv) * d)),
                (p + "self_attn.v_proj.weight", *row_slice(L.qkv_weight, (nh + nkv) * d, (nh + 2 * nkv) * d)),
                (p + "self_attn.o_proj.weight", *whole(L.o_weight)),
                (p + "mlp.gate_proj.weight", *row_slice(L.gate_up_weight, 0, I)),
                (p + "mlp.up_proj.weight", *row_slice(L.gate_up_weight, I, 2 * I)),
                (p + "mlp.down_proj.weight", *whole(L.down_weight)),
                (p + "input_layernorm.weight", *whole(L.in_ln)),
                (p + "post_attention_layernorm.weight", *whole(L.post_ln)),
            ]
        it += [("model.norm.weight", *whole(self.norm)), ("score.weight", *whole(self.score_weight))]
        return it

    def adapter_items(self):
        """PEFT-style names of the trainable (exchanged) tensors only."""
        it = []
        c = self.cfg
        r = c.lora_rank
        if self.lora:
            for i, L in enumerate(self.layers):
                p = f"base_model.model.model.layers.{i}."
                for lora, names in ((L.lora_qkv, ("self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj")),
                                    (L.lora_o, ("self_attn.o_proj",)),
                                    (L.lora_gate_up, ("mlp.gate_proj", "mlp.up_proj")),
                                    (L.lora_down, ("mlp.down_proj",))):
                    for j, nm in enumerate(names):
                        it.append((p + nm + ".lora_A.weight", *row_slice(lora.A, j * r, (j + 1) * r)))
                        it.append((p + nm + ".lora_B.weight", *whole(lora.B[j])))
        it.append(("base_model.model.score.weight", *whole(self.score_weight)))
        return it

    def hf_config(self) -> Dict:
        c = self.cfg
        return dict(architectures=[self.hf_architecture], model_type="llama",
                    vocab_size=c.vocab_size, hidden_size=c.hidden_size,
                    intermediate_size=c.intermediate_size, num_hidden_layers=c.num_hidden_layers,
                    num_attention_heads=c.num_attention_heads,
                    num_key_value_heads=c.num_key_value_heads,
                    max_position_embeddings=c.max_position_embeddings, rms_norm_eps=c.rms_norm_eps,
                    rope_theta=c.rope_theta, hidden_act="silu", tie_word_embeddings=False,
                    attention_bias=False, mlp_bias=False, pad_token_id=c.pad_token_id,
                    bos_token_id=c.cls_token_id, eos_token_id=c.sep_token_id,
                    id2label={str(i): f"LABEL_{i}" for i in range(c.num_labels)},
                    label2id={f"LABEL_{i}": i for i in range(c.num_labels)},
                    torch_dtype="bfloat16")
