"""BERT / BioBERT for sequence classification on packed (varlen) batches.

Same architecture and HF state-dict names as ``transformers.BertForSequenceClassification``
(the reference loads it via ``AutoModelForSequenceClassification.from_pretrained`` at
``src/Servercase/server_IID_IMDB.py:142-144``; architecture print-out at
``serverless_cancer_classification_with_BioBERT.ipynb:526-569``), re-laid-out for MI355X:

* Q, K, V projections are ONE fused [3H, H] weight (one hipBLASLt GEMM, N = 2304) whose row blocks
  are exported under the HF names ``attention.self.{query,key,value}``.
* Dense-layer biases are NOT applied by the GEMM where a fused epilogue kernel follows: the
  attention-output / FFN-output biases go into the bias+dropout+residual+LayerNorm kernel and the
  intermediate bias into the bias+GELU kernel.
* Activations are packed rows ``[T, H]`` (T = valid tokens only); attention is varlen flash
  attention over ``cu_seqlens`` — padding is never computed.
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
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    layer_norm_eps: float = 1e-12
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    classifier_dropout: Optional[float] = None
    num_labels: int = 2
    hidden_act: str = "gelu"
    pad_token_id: int = 0
    initializer_range: float = 0.02
    cls_token_id: int = 101
    sep_token_id: int = 102

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads


class BertLayer(nn.Module):
    def __init__(self, cfg: BertConfig, device=None, dtype=torch.float32):
        super().__init__()
        H, I, std = cfg.hidden_size, cfg.intermediate_size, cfg.initializer_range
        self.cfg = cfg
        self.qkv_weight = new_param((3 * H, H), device, dtype, "normal", std)
        self.qkv_bias = new_param((3 * H,), device, dtype, "zeros")
        self.attn_out_weight = new_param((H, H), device, dtype, "normal", std)
        self.attn_out_bias = new_param((H,), device, dtype, "zeros")
        self.attn_ln_weight = new_param((H,), device, dtype, "ones")
        self.attn_ln_bias = new_param((H,), device, dtype, "zeros")
        self.inter_weight = new_param((I, H), device, dtype, "normal", std)
        self.inter_bias = new_param((I,), device, dtype, "zeros")
        self.out_weight = new_param((H, I), device, dtype, "normal", std)
        self.out_bias = new_param((H,), device, dtype, "zeros")
        self.out_ln_weight = new_param((H,), device, dtype, "ones")
        self.out_ln_bias = new_param((H,), device, dtype, "zeros")

    def forward(self, x: torch.Tensor, batch: PackedBatch,
                rows: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``rows``: compute the layer's output only for these token rows (the pooled [CLS] rows
        of the last layer; K and V still come from every token)."""
        c = self.cfg
        tr = self.training
        # the residual gradients of both LayerNorms go straight into the dgrad GEMMs that read
        # the same tensors (no separate gradient-sum pass; ops.ResidualTap)
        t_attn, t_ffn = ops.ResidualTap(), ops.ResidualTap()
        qkv = ops.linear(x, self.qkv_weight, self.qkv_bias, tap=t_attn if rows is None else None)
        if rows is None:
            ctx = ops.varlen_attention(qkv, batch.cu_seqlens, batch.cu_host, batch.max_seqlen,
                                       c.num_attention_heads, c.num_attention_heads, c.head_dim,
                                       c.attention_probs_dropout_prob, tr,
                                       sched=getattr(batch, "attn_sched", None))
        else:
            ctx = ops.query_subset_attention(qkv, rows, batch.cu_seqlens, batch.max_seqlen,
                                             c.num_attention_heads, c.num_attention_heads,
                                             c.head_dim, c.attention_probs_dropout_prob, tr)
            x = x.index_select(0, rows.long())
        y = ops.linear(ctx, self.attn_out_weight)
        x1 = ops.bias_dropout_add_layernorm(y, self.attn_out_bias, x, self.attn_ln_weight,
                                            self.attn_ln_bias, c.layer_norm_eps,
                                            c.hidden_dropout_prob, tr, tap=t_attn)
        # dense -> GELU in one GEMM epilogue; the output GEMM's backward applies GELU' (K6)
        h, pre = ops.linear_act(x1, self.inter_weight, self.inter_bias, c.hidden_act, tap=t_ffn)
        y2 = ops.linear_after_act(h, pre, self.out_weight, c.hidden_act)
        return ops.bias_dropout_add_layernorm(y2, self.out_bias, x1, self.out_ln_weight,
                                              self.out_ln_bias, c.layer_norm_eps,
                                              c.hidden_dropout_prob, tr, tap=t_ffn)

    def hf_items(self, prefix: str):
        H = self.cfg.hidden_size
        it = []
        for j, nm in enumerate(("query", "key", "value")):
            it.append((f"{prefix}attention.self.{nm}.weight", *row_slice(self.qkv_weight, j * H, (j + 1) * H)))
            it.append((f"{prefix}attention.self.{nm}.bias", *row_slice(self.qkv_bias, j * H, (j + 1) * H)))
        it += [
            (f"{prefix}attention.output.dense.weight", *whole(self.attn_out_weight)),
            (f"{prefix}attention.output.dense.bias", *whole(self.attn_out_bias)),
            (f"{prefix}attention.output.LayerNorm.weight", *whole(self.attn_ln_weight)),
            (f"{prefix}attention.output.LayerNorm.bias", *whole(self.attn_ln_bias)),
            (f"{prefix}intermediate.dense.weight", *whole(self.inter_weight)),
            (f"{prefix}intermediate.dense.bias", *whole(self.inter_bias)),
            (f"{prefix}output.dense.weight", *whole(self.out_weight)),
            (f"{prefix}output.dense.bias", *whole(self.out_bias)),
            (f"{prefix}output.LayerNorm.weight", *whole(self.out_ln_weight)),
            (f"{prefix}output.LayerNorm.bias", *whole(self.out_ln_bias)),
        ]
        return it


class BertForSequenceClassification(SeqClassifierBase):
    hf_architecture = "BertForSequenceClassification"
    hf_model_type = "bert"

    def __init__(self, cfg: BertConfig, device=None, dtype=torch.float32):
        super().__init__()
        H, std = cfg.hidden_size, cfg.initializer_range
        self.cfg = cfg
        self.word_embeddings = new_param((cfg.vocab_size, H), device, dtype, "normal", std)
        self.position_embeddings = new_param((cfg.max_position_embeddings, H), device, dtype, "normal", std)
        self.token_type_embeddings = new_param((cfg.type_vocab_size, H), device, dtype, "normal", std)
        with torch.no_grad():
            self.word_embeddings[cfg.pad_token_id].zero_()
        self.emb_ln_weight = new_param((H,), device, dtype, "ones")
        self.emb_ln_bias = new_param((H,), device, dtype, "zeros")
        self.layers = nn.ModuleList([BertLayer(cfg, device, dtype) for _ in range(cfg.num_hidden_layers)])
        self.pooler_weight = new_param((H, H), device, dtype, "normal", std)
        self.pooler_bias = new_param((H,), device, dtype, "zeros")
        self.classifier_weight = new_param((cfg.num_labels, H), device, dtype, "normal", std)
        self.classifier_bias = new_param((cfg.num_labels,), device, dtype, "zeros")

    def encode(self, batch: PackedBatch, token_type_ids: Optional[torch.Tensor] = None,
               rows: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Hidden states of every token ([T, H]); with ``rows``, the last layer only produces
        those rows ([len(rows), H])."""
        c = self.cfg
        check_positions(batch, c.max_position_embeddings)
        x = ops.embedding_layernorm(batch.input_ids, batch.position_ids, token_type_ids,
                                    self.word_embeddings, self.position_embeddings,
                                    self.token_type_embeddings, self.emb_ln_weight,
                                    self.emb_ln_bias, c.layer_norm_eps, c.hidden_dropout_prob,
                                    self.training, order=batch.order())
        last = len(self.layers) - 1
        for i, layer in enumerate(self.layers):
            x = layer(x, batch, rows if i == last else None)
        return x

    def forward(self, batch: PackedBatch, token_type_ids: Optional[torch.Tensor] = None) -> torch.Tensor:
        c = self.cfg
        rows = batch.cu_seqlens[:batch.n_seq]
        if self.pooled_rows_only:
            cls = self.encode(batch, token_type_ids, rows)
        else:
            cls = self.encode(batch, token_type_ids).index_select(0, rows.long())
        pooled = torch.tanh(ops.linear(cls, self.pooler_weight, self.pooler_bias))
        p = c.classifier_dropout if c.classifier_dropout is not None else c.hidden_dropout_prob
        if self.training and p > 0:
            pooled = ops.dropout(pooled, p, True)
        return ops.linear(pooled, self.classifier_weight, self.classifier_bias)

    def hf_items(self):
        it = [
            ("bert.embeddings.word_embeddings.weight", *whole(self.word_embeddings)),
            ("bert.embeddings.position_embeddings.weight", *whole(self.position_embeddings)),
            ("bert.embeddings.token_type_embeddings.weight", *whole(self.token_type_embeddings)),
            ("bert.embeddings.LayerNorm.weight", *whole(self.emb_ln_weight)),
            ("bert.embeddings.LayerNorm.bias", *whole(self.emb_ln_bias)),
        ]
        for i, layer in enumerate(self.layers):
            it += layer.hf_items(f"bert.encoder.layer.{i}.")
        it += [
            ("bert.pooler.dense.weight", *whole(self.pooler_weight)),
            ("bert.pooler.dense.bias", *whole(self.pooler_bias)),
            ("classifier.weight", *whole(self.classifier_weight)),
            ("classifier.bias", *whole(self.classifier_bias)),
        ]
        return it

    def hf_config(self) -> Dict:
        c = asdict(self.cfg)
        for k in ("cls_token_id", "sep_token_id"):
            c.pop(k)
        c.update(architectures=[self.hf_architecture], model_type=self.hf_model_type,
                 id2label={str(i): f"LABEL_{i}" for i in range(self.cfg.num_labels)},
                 label2id={f"LABEL_{i}": i for i in range(self.cfg.num_labels)},
                 position_embedding_type="absolute", torch_dtype="float32")
        c.pop("num_labels")
        return c
