"""ALBERT (albert-base-v2) for sequence classification on packed batches.

Reference usage: ``CHECKPOINT = "albert-base-v2"`` in ``src/Serverlesscase/serverless_IID_IMDB.py:31``
and the other ALBERT scripts. Differences from BERT: factorised embeddings
(E=128) with a 128->768 mapping, ONE shared transformer layer applied ``num_hidden_layers`` times
(its weight gradients accumulate 12x into the same flat-buffer slots), ``gelu_new`` activation,
and hidden/attention dropout 0 with classifier dropout 0.1. HF names: 27 tensors.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass
from typing import Dict, Optional

import torch
import torch.nn as nn

from .. import ops
from ..data.batching import PackedBatch
from .common import SeqClassifierBase, new_param, row_slice, whole, check_positions


@dataclass
class AlbertConfig:
    vocab_size: int = 30000
    embedding_size: int = 128
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    layer_norm_eps: float = 1e-12
    hidden_dropout_prob: float = 0.0
    attention_probs_dropout_prob: float = 0.0
    classifier_dropout_prob: float = 0.1
    num_labels: int = 2
    hidden_act: str = "gelu_new"
    pad_token_id: int = 0
    initializer_range: float = 0.02
    cls_token_id: int = 2
    sep_token_id: int = 3

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads


class AlbertForSequenceClassification(SeqClassifierBase):
    hf_architecture = "AlbertForSequenceClassification"
    hf_model_type = "albert"

    def __init__(self, cfg: AlbertConfig, device=None, dtype=torch.float32):
        super().__init__()
        E, H, I, std = cfg.embedding_size, cfg.hidden_size, cfg.intermediate_size, cfg.initializer_range
        self.cfg = cfg
        self.word_embeddings = new_param((cfg.vocab_size, E), device, dtype, "normal", std)
        self.position_embeddings = new_param((cfg.max_position_embeddings, E), device, dtype, "normal", std)
        self.token_type_embeddings = new_param((cfg.type_vocab_size, E), device, dtype, "normal", std)
        with torch.no_grad():
            self.word_embeddings[cfg.pad_token_id].zero_()
        self.emb_ln_weight = new_param((E,), device, dtype, "ones")
        self.emb_ln_bias = new_param((E,), device, dtype, "zeros")
        self.map_weight = new_param((H, E), device, dtype, "normal", std)
        self.map_bias = new_param((H,), device, dtype, "zeros")
        # the ONE shared layer
        self.full_ln_weight = new_param((H,), device, dtype, "ones")
        self.full_ln_bias = new_param((H,), device, dtype, "zeros")
        self.qkv_weight = new_param((3 * H, H), device, dtype, "normal", std)
        self.qkv_bias = new_param((3 * H,), device, dtype, "zeros")
        self.dense_weight = new_param((H, H), device, dtype, "normal", std)
        self.dense_bias = new_param((H,), device, dtype, "zeros")
        self.attn_ln_weight = new_param((H,), device, dtype, "ones")
        self.attn_ln_bias = new_param((H,), device, dtype, "zeros")
        self.ffn_weight = new_param((I, H), device, dtype, "normal", std)
        self.ffn_bias = new_param((I,), device, dtype, "zeros")
        self.ffn_out_weight = new_param((H, I), device, dtype, "normal", std)
        self.ffn_out_bias = new_param((H,), device, dtype, "zeros")
        self.pooler_weight = new_param((H, H), device, dtype, "normal", std)
        self.pooler_bias = new_param((H,), device, dtype, "zeros")
        self.classifier_weight = new_param((cfg.num_labels, H), device, dtype, "normal", std)
        self.classifier_bias = new_param((cfg.num_labels,), device, dtype, "zeros")
        # applied num_hidden_layers times: autograd sums their gradients, so their weight
        # gradients must stay on autograd's stream (no side-stream overlap)
        for p in (self.qkv_weight, self.qkv_bias, self.dense_weight, self.dense_bias,
                  self.ffn_weight, self.ffn_bias, self.ffn_out_weight, self.ffn_out_bias):
            p._bcfl_shared = True

    def _layer(self, x, batch, rows=None):
        c, tr = self.cfg, self.training
        t_attn, t_ffn = ops.ResidualTap(), ops.ResidualTap()   # see BertLayer.forward
        qkv = ops.linear(x, self.qkv_weight, self.qkv_bias, tap=t_attn if rows is None else None)
        if rows is None:
            ctx = ops.varlen_attention(qkv, batch.cu_seqlens, batch.cu_host, batch.max_seqlen,
                                       c.num_attention_heads, c.num_attention_heads, c.head_dim,
                                       c.attention_probs_dropout_prob, tr,
                                       sched=getattr(batch, "attn_sched", None))
        else:  # last application: only the pooled [CLS] rows are consumed
            ctx = ops.query_subset_attention(qkv, rows, batch.cu_seqlens, batch.max_seqlen,
                                             c.num_attention_heads, c.num_attention_heads,
                                             c.head_dim, c.attention_probs_dropout_prob, tr)
            x = x.index_select(0, rows.long())
        x1 = ops.bias_dropout_add_layernorm(ops.linear(ctx, self.dense_weight), self.dense_bias, x,
                                            self.attn_ln_weight, self.attn_ln_bias,
                                            c.layer_norm_eps, c.hidden_dropout_prob, tr, tap=t_attn)
        h, pre = ops.linear_act(x1, self.ffn_weight, self.ffn_bias, c.hidden_act, tap=t_ffn)
        y2 = ops.linear_after_act(h, pre, self.ffn_out_weight, c.hidden_act)
        return ops.bias_dropout_add_layernorm(y2, self.ffn_out_bias,
                                              x1, self.full_ln_weight, self.full_ln_bias,
                                              c.layer_norm_eps, 0.0, tr, tap=t_ffn)

    def forward(self, batch: PackedBatch, token_type_ids: Optional[torch.Tensor] = None):
        c = self.cfg
        check_positions(batch, c.max_position_embeddings)
        e = ops.embedding_layernorm(batch.input_ids, batch.position_ids, token_type_ids,
                                    self.word_embeddings, self.position_embeddings,
                                    self.token_type_embeddings, self.emb_ln_weight,
                                    self.emb_ln_bias, c.layer_norm_eps, c.hidden_dropout_prob,
                                    self.training, order=batch.order())
        x = ops.linear(e, self.map_weight, self.map_bias)
        rows = batch.cu_seqlens[:batch.n_seq]
        for i in range(c.num_hidden_layers):
            last = i == c.num_hidden_layers - 1 and self.pooled_rows_only
            x = self._layer(x, batch, rows if last else None)
        cls = x if self.pooled_rows_only else x.index_select(0, rows.long())
        pooled = torch.tanh(ops.linear(cls, self.pooler_weight, self.pooler_bias))
        if self.training and c.classifier_dropout_prob > 0:
            pooled = ops.dropout(pooled, c.classifier_dropout_prob, True)
        return ops.linear(pooled, self.classifier_weight, self.classifier_bias)

    def hf_items(self):
        H = self.cfg.hidden_size
        L = "albert.encoder.albert_layer_groups.0.albert_layers.0."
        it = [
            ("albert.embeddings.word_embeddings.weight", *whole(self.word_embeddings)),
            ("albert.embeddings.position_embeddings.weight", *whole(self.position_embeddings)),
            ("albert.embeddings.token_type_embeddings.weight", *whole(self.token_type_embeddings)),
            ("albert.embeddings.LayerNorm.weight", *whole(self.emb_ln_weight)),
            ("albert.embeddings.LayerNorm.bias", *whole(self.emb_ln_bias)),
            ("albert.encoder.embedding_hidden_mapping_in.weight", *whole(self.map_weight)),
            ("albert.encoder.embedding_hidden_mapping_in.bias", *whole(self.map_bias)),
            (L + "full_layer_layer_norm.weight", *whole(self.full_ln_weight)),
            (L + "full_layer_layer_norm.bias", *whole(self.full_ln_bias)),
        ]
        for j, nm in enumerate(("query", "key", "value")):
            it.append((L + f"attention.{nm}.weight", *row_slice(self.qkv_weight, j * H, (j + 1) * H)))
            it.append((L + f"attention.{nm}.bias", *row_slice(self.qkv_bias, j * H, (j + 1) * H)))
        it += [
            (L + "attention.dense.weight", *whole(self.dense_weight)),
            (L + "attention.dense.bias", *whole(self.dense_bias)),
            (L + "attention.LayerNorm.weight", *whole(self.attn_ln_weight)),
            (L + "attention.LayerNorm.bias", *whole(self.attn_ln_bias)),
            (L + "ffn.weight", *whole(self.ffn_weight)),
            (L + "ffn.bias", *whole(self.ffn_bias)),
            (L + "ffn_output.weight", *whole(self.ffn_out_weight)),
            (L + "ffn_output.bias", *whole(self.ffn_out_bias)),
            ("albert.pooler.weight", *whole(self.pooler_weight)),
            ("albert.pooler.bias", *whole(self.pooler_bias)),
            ("classifier.weight", *whole(self.classifier_weight)),
            ("classifier.bias", *whole(self.classifier_bias)),
        ]
        return it

    def hf_config(self) -> Dict:
        c = asdict(self.cfg)
        for k in ("cls_token_id", "sep_token_id", "num_labels"):
            c.pop(k)
        c.update(architectures=[self.hf_architecture], model_type=self.hf_model_type,
                 num_hidden_groups=1, inner_group_num=1,
                 id2label={str(i): f"LABEL_{i}" for i in range(self.cfg.num_labels)},
                 label2id={f"LABEL_{i}": i for i in range(self.cfg.num_labels)},
                 position_embedding_type="absolute", torch_dtype="float32")
        return c
