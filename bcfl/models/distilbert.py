"""DistilBERT for sequence classification (BASELINE.json config 1; not used by the reference).

6 layers, no token-type embedding, head = pre_classifier -> ReLU -> dropout(0.2) -> classifier.
HF names (104 tensors): ``distilbert.transformer.layer.{i}.attention.{q,k,v,out}_lin``,
``sa_layer_norm``, ``ffn.lin1``, ``ffn.lin2``, ``output_layer_norm``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import torch
import torch.nn as nn

from .. import ops
from ..data.batching import PackedBatch
from .common import SeqClassifierBase, new_param, row_slice, whole, check_positions


@dataclass
class DistilBertConfig:
    vocab_size: int = 30522
    dim: int = 768
    n_layers: int = 6
    n_heads: int = 12
    hidden_dim: int = 3072
    max_position_embeddings: int = 512
    dropout: float = 0.1
    attention_dropout: float = 0.1
    seq_classif_dropout: float = 0.2
    num_labels: int = 2
    activation: str = "gelu"
    pad_token_id: int = 0
    initializer_range: float = 0.02
    layer_norm_eps: float = 1e-12
    cls_token_id: int = 101
    sep_token_id: int = 102

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads


class DistilBertLayer(nn.Module):
    def __init__(self, cfg: DistilBertConfig, device=None, dtype=torch.float32):
        super().__init__()
        H, I, std = cfg.dim, cfg.hidden_dim, cfg.initializer_range
        self.cfg = cfg
        self.qkv_weight = new_param((3 * H, H), device, dtype, "normal", std)
        self.qkv_bias = new_param((3 * H,), device, dtype, "zeros")
        self.out_lin_weight = new_param((H, H), device, dtype, "normal", std)
        self.out_lin_bias = new_param((H,), device, dtype, "zeros")
        self.sa_ln_weight = new_param((H,), device, dtype, "ones")
        self.sa_ln_bias = new_param((H,), device, dtype, "zeros")
        self.lin1_weight = new_param((I, H), device, dtype, "normal", std)
        self.lin1_bias = new_param((I,), device, dtype, "zeros")
        self.lin2_weight = new_param((H, I), device, dtype, "normal", std)
        self.lin2_bias = new_param((H,), device, dtype, "zeros")
        self.out_ln_weight = new_param((H,), device, dtype, "ones")
        self.out_ln_bias = new_param((H,), device, dtype, "zeros")

    def forward(self, x, batch: PackedBatch, rows=None):
        c, tr = self.cfg, self.training
        t_attn, t_ffn = ops.ResidualTap(), ops.ResidualTap()   # see BertLayer.forward
        qkv = ops.linear(x, self.qkv_weight, self.qkv_bias, tap=t_attn if rows is None else None)
        if rows is None:
            ctx = ops.varlen_attention(qkv, batch.cu_seqlens, batch.cu_host, batch.max_seqlen,
                                       c.n_heads, c.n_heads, c.head_dim, c.attention_dropout, tr,
                                       sched=getattr(batch, "attn_sched", None))
        else:  # last layer: only the pooled [CLS] rows are consumed
            ctx = ops.query_subset_attention(qkv, rows, batch.cu_seqlens, batch.max_seqlen,
                                             c.n_heads, c.n_heads, c.head_dim,
                                             c.attention_dropout, tr)
            x = x.index_select(0, rows.long())
        x1 = ops.bias_dropout_add_layernorm(ops.linear(ctx, self.out_lin_weight), self.out_lin_bias,
                                            x, self.sa_ln_weight, self.sa_ln_bias,
                                            c.layer_norm_eps, 0.0, tr, tap=t_attn)
        h, pre = ops.linear_act(x1, self.lin1_weight, self.lin1_bias, c.activation, tap=t_ffn)
        y2 = ops.linear_after_act(h, pre, self.lin2_weight, c.activation)
        return ops.bias_dropout_add_layernorm(y2, self.lin2_bias, x1,
                                              self.out_ln_weight, self.out_ln_bias,
                                              c.layer_norm_eps, c.dropout, tr, tap=t_ffn)

    def hf_items(self, prefix):
        H = self.cfg.dim
        it = []
        for j, nm in enumerate(("q_lin", "k_lin", "v_lin")):
            it.append((f"{prefix}attention.{nm}.weight", *row_slice(self.qkv_weight, j * H, (j + 1) * H)))
            it.append((f"{prefix}attention.{nm}.bias", *row_slice(self.qkv_bias, j * H, (j + 1) * H)))
        it += [
            (f"{prefix}attention.out_lin.weight", *whole(self.out_lin_weight)),
            (f"{prefix}attention.out_lin.bias", *whole(self.out_lin_bias)),
            (f"{prefix}sa_layer_norm.weight", *whole(self.sa_ln_weight)),
            (f"{prefix}sa_layer_norm.bias", *whole(self.sa_ln_bias)),
            (f"{prefix}ffn.lin1.weight", *whole(self.lin1_weight)),
            (f"{prefix}ffn.lin1.bias", *whole(self.lin1_bias)),
            (f"{prefix}ffn.lin2.weight", *whole(self.lin2_weight)),
            (f"{prefix}ffn.lin2.bias", *whole(self.lin2_bias)),
            (f"{prefix}output_layer_norm.weight", *whole(self.out_ln_weight)),
            (f"{prefix}output_layer_norm.bias", *whole(self.out_ln_bias)),
        ]
        return it


class DistilBertForSequenceClassification(SeqClassifierBase):
    hf_architecture = "DistilBertForSequenceClassification"
    hf_model_type = "distilbert"

    def __init__(self, cfg: DistilBertConfig, device=None, dtype=torch.float32):
        super().__init__()
        H, std = cfg.dim, cfg.initializer_range
        self.cfg = cfg
        self.word_embeddings = new_param((cfg.vocab_size, H), device, dtype, "normal", std)
        self.position_embeddings = new_param((cfg.max_position_embeddings, H), device, dtype, "normal", std)
        with torch.no_grad():
            self.word_embeddings[cfg.pad_token_id].zero_()
        self.emb_ln_weight = new_param((H,), device, dtype, "ones")
        self.emb_ln_bias = new_param((H,), device, dtype, "zeros")
        self.layers = nn.ModuleList([DistilBertLayer(cfg, device, dtype) for _ in range(cfg.n_layers)])
        self.pre_classifier_weight = new_param((H, H), device, dtype, "normal", std)
        self.pre_classifier_bias = new_param((H,), device, dtype, "zeros")
        self.classifier_weight = new_param((cfg.num_labels, H), device, dtype, "normal", std)
        self.classifier_bias = new_param((cfg.num_labels,), device, dtype, "zeros")

    def forward(self, batch: PackedBatch, token_type_ids: Optional[torch.Tensor] = None):
        c = self.cfg
        check_positions(batch, c.max_position_embeddings)
        x = ops.embedding_layernorm(batch.input_ids, batch.position_ids, None, self.word_embeddings,
                                    self.position_embeddings, None, self.emb_ln_weight,
                                    self.emb_ln_bias, c.layer_norm_eps, c.dropout, self.training, order=batch.order())
        rows = batch.cu_seqlens[:batch.n_seq]
        last = len(self.layers) - 1
        for i, layer in enumerate(self.layers):
            x = layer(x, batch, rows if (i == last and self.pooled_rows_only) else None)
        cls = x if self.pooled_rows_only else x.index_select(0, rows.long())
        h = torch.relu(ops.linear(cls, self.pre_classifier_weight, self.pre_classifier_bias))
        if self.training and c.seq_classif_dropout > 0:
            h = ops.dropout(h, c.seq_classif_dropout, True)
        return ops.linear(h, self.classifier_weight, self.classifier_bias)

    def hf_items(self):
        it = [
            ("distilbert.embeddings.word_embeddings.weight", *whole(self.word_embeddings)),
            ("distilbert.embeddings.position_embeddings.weight", *whole(self.position_embeddings)),
            ("distilbert.embeddings.LayerNorm.weight", *whole(self.emb_ln_weight)),
            ("distilbert.embeddings.LayerNorm.bias", *whole(self.emb_ln_bias)),
        ]
        for i, layer in enumerate(self.layers):
            it += layer.hf_items(f"distilbert.transformer.layer.{i}.")
        it += [
            ("pre_classifier.weight", *whole(self.pre_classifier_weight)),
            ("pre_classifier.bias", *whole(self.pre_classifier_bias)),
            ("classifier.weight", *whole(self.classifier_weight)),
            ("classifier.bias", *whole(self.classifier_bias)),
        ]
        return it

    def hf_config(self) -> Dict:
        c = self.cfg
        return dict(architectures=[self.hf_architecture], model_type=self.hf_model_type,
                    vocab_size=c.vocab_size, dim=c.dim, n_layers=c.n_layers, n_heads=c.n_heads,
                    hidden_dim=c.hidden_dim, max_position_embeddings=c.max_position_embeddings,
                    dropout=c.dropout, attention_dropout=c.attention_dropout,
                    seq_classif_dropout=c.seq_classif_dropout, activation=c.activation,
                    pad_token_id=c.pad_token_id, initializer_range=c.initializer_range,
                    id2label={str(i): f"LABEL_{i}" for i in range(c.num_labels)},
                    label2id={f"LABEL_{i}": i for i in range(c.num_labels)},
                    sinusoidal_pos_embds=False, qa_dropout=0.1, tie_weights_=True,
                    torch_dtype="float32")
