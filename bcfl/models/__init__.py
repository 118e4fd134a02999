"""Model registry. Names follow the reference's ``CHECKPOINT`` ids."""
from __future__ import annotations

from dataclasses import replace
from typing import Optional

import torch

from .albert import AlbertConfig, AlbertForSequenceClassification
from .bert import BertConfig, BertForSequenceClassification
from .common import SeqClassifierBase, padded_to_packed
from .distilbert import DistilBertConfig, DistilBertForSequenceClassification
from .llama import LlamaConfig, LlamaForSequenceClassification

MODEL_CONFIGS = {
    # bert-base-uncased
    "bert-base": (BertForSequenceClassification, BertConfig()),
    # dmis-lab/biobert-v1.1 (BERT-base cased, vocab 28996; 108.34 M params @ 41 labels)
    "biobert": (BertForSequenceClassification, BertConfig(vocab_size=28996)),
    "albert-base-v2": (AlbertForSequenceClassification, AlbertConfig()),
    "distilbert": (DistilBertForSequenceClassification, DistilBertConfig()),
    "llama3-8b-lora": (LlamaForSequenceClassification, LlamaConfig()),
    # tiny variants for tests / CPU plumbing
    "tiny-bert": (BertForSequenceClassification,
                  BertConfig(vocab_size=2048, hidden_size=64, num_hidden_layers=2,
                             num_attention_heads=2, intermediate_size=128,
                             max_position_embeddings=128)),
    "tiny-albert": (AlbertForSequenceClassification,
                    AlbertConfig(vocab_size=2048, embedding_size=32, hidden_size=64,
                                 num_hidden_layers=3, num_attention_heads=2,
                                 intermediate_size=128, max_position_embeddings=128)),
    "tiny-distilbert": (DistilBertForSequenceClassification,
                        DistilBertConfig(vocab_size=2048, dim=64, n_layers=2, n_heads=2,
                                         hidden_dim=128, max_position_embeddings=128)),
    "tiny-llama-lora": (LlamaForSequenceClassification,
                        LlamaConfig(vocab_size=2048, hidden_size=128, intermediate_size=256,
                                    num_hidden_layers=2, num_attention_heads=4,
                                    num_key_value_heads=2, max_position_embeddings=256,
                                    lora_rank=4, lora_alpha=8.0, cls_token_id=1,
                                    sep_token_id=2, pad_token_id=0)),
    # BERT-base geometry, 2 layers: GPU kernel smoke tests at the real head_dim / hidden size
    "bert-base-2l": (BertForSequenceClassification, BertConfig(num_hidden_layers=2)),
}


def model_config(name: str, num_labels: Optional[int] = None, dropout: Optional[float] = None,
                 vocab_size: Optional[int] = None, lora_rank: Optional[int] = None,
                 lora_alpha: Optional[float] = None):
    if name not in MODEL_CONFIGS:
        raise KeyError(f"unknown model {name!r}; known {sorted(MODEL_CONFIGS)}")
    cls, cfg = MODEL_CONFIGS[name]
    kw = {}
    if num_labels is not None:
        kw["num_labels"] = num_labels
    if vocab_size is not None:
        kw["vocab_size"] = vocab_size
    if dropout is not None:
        if isinstance(cfg, BertConfig):
            kw.update(hidden_dropout_prob=dropout, attention_probs_dropout_prob=dropout)
        elif isinstance(cfg, AlbertConfig):
            kw.update(hidden_dropout_prob=dropout, attention_probs_dropout_prob=dropout,
                      classifier_dropout_prob=dropout)
        elif isinstance(cfg, DistilBertConfig):
            kw.update(dropout=dropout, attention_dropout=dropout, seq_classif_dropout=dropout)
    if isinstance(cfg, LlamaConfig):
        if lora_rank is not None:
            kw["lora_rank"] = lora_rank
        if lora_alpha is not None:
            kw["lora_alpha"] = lora_alpha
    return cls, replace(cfg, **kw)


def build_model(name: str, num_labels: Optional[int] = None, device=None,
                dtype: torch.dtype = torch.float32, dropout: Optional[float] = None,
                vocab_size: Optional[int] = None, seed: Optional[int] = None, **kw) -> SeqClassifierBase:
    cls, cfg = model_config(name, num_labels, dropout, vocab_size, kw.get("lora_rank"),
                            kw.get("lora_alpha"))
    if seed is not None:
        torch.manual_seed(seed)
    if cls is LlamaForSequenceClassification:
        return cls(cfg, device=device, dtype=dtype, lora=name.endswith("lora"))
    return cls(cfg, device=device, dtype=dtype)


def special_tokens(name: str):
    _, cfg = model_config(name)
    return cfg.cls_token_id, cfg.sep_token_id, cfg.vocab_size


__all__ = ["MODEL_CONFIGS", "model_config", "build_model", "special_tokens", "SeqClassifierBase",
           "padded_to_packed", "BertConfig", "BertForSequenceClassification", "AlbertConfig",
           "AlbertForSequenceClassification", "DistilBertConfig",
           "DistilBertForSequenceClassification", "LlamaConfig", "LlamaForSequenceClassification"]
