"""Model parity with transformers (same weights -> same logits) and HF state-dict layouts."""
import numpy as np
import pytest
import torch

from bcfl.data.batching import make_padded_batch
from bcfl.data.registry import load_split
from bcfl.models import build_model

transformers = pytest.importorskip("transformers")


def _batch(vocab, max_len=128, n=6):
    ds = load_split("tiny", "train", vocab, max_len)
    return make_padded_batch(ds, np.arange(0, 6 * n, 6)[:n])


def _load(hf, ours):
    sd = ours.hf_state_dict()
    missing, unexpected = hf.load_state_dict(dict(sd), strict=False)
    assert not unexpected
    assert all("position_ids" in k or "token_type_ids" in k for k in missing), missing


def test_bert_parity():
    m = build_model("tiny-bert", num_labels=3, seed=0).eval()
    c = m.cfg
    hf = transformers.BertForSequenceClassification(transformers.BertConfig(
        vocab_size=c.vocab_size, hidden_size=c.hidden_size, num_hidden_layers=c.num_hidden_layers,
        num_attention_heads=c.num_attention_heads, intermediate_size=c.intermediate_size,
        max_position_embeddings=c.max_position_embeddings, num_labels=3)).eval()
    _load(hf, m)
    b = _batch(c.vocab_size)
    with torch.no_grad():
        ours = m.forward_padded(b.input_ids, b.attention_mask)
        ref = hf(input_ids=b.input_ids, attention_mask=b.attention_mask).logits
    torch.testing.assert_close(ours, ref, atol=2e-5, rtol=1e-4)


def test_albert_parity():
    m = build_model("tiny-albert", num_labels=2, seed=0).eval()
    c = m.cfg
    hf = transformers.AlbertForSequenceClassification(transformers.AlbertConfig(
        vocab_size=c.vocab_size, embedding_size=c.embedding_size, hidden_size=c.hidden_size,
        num_hidden_layers=c.num_hidden_layers, num_attention_heads=c.num_attention_heads,
        intermediate_size=c.intermediate_size, max_position_embeddings=c.max_position_embeddings,
        hidden_act="gelu_new", num_labels=2, hidden_dropout_prob=0.0,
        attention_probs_dropout_prob=0.0)).eval()
    _load(hf, m)
    b = _batch(c.vocab_size)
    with torch.no_grad():
        ours = m.forward_padded(b.input_ids, b.attention_mask)
        ref = hf(input_ids=b.input_ids, attention_mask=b.attention_mask).logits
    torch.testing.assert_close(ours, ref, atol=2e-5, rtol=1e-4)


def test_distilbert_parity():
    m = build_model("tiny-distilbert", num_labels=2, seed=0).eval()
    c = m.cfg
    hf = transformers.DistilBertForSequenceClassification(transformers.DistilBertConfig(
        vocab_size=c.vocab_size, dim=c.dim, n_layers=c.n_layers, n_heads=c.n_heads,
        hidden_dim=c.hidden_dim, max_position_embeddings=c.max_position_embeddings,
        num_labels=2)).eval()
    _load(hf, m)
    b = _batch(c.vocab_size)
    with torch.no_grad():
        ours = m.forward_padded(b.input_ids, b.attention_mask)
        ref = hf(input_ids=b.input_ids, attention_mask=b.attention_mask).logits
    torch.testing.assert_close(ours, ref, atol=2e-5, rtol=1e-4)


def test_llama_parity_base_weights():
    m = build_model("tiny-llama-lora", num_labels=2, seed=0, dtype=torch.float32).eval()
    c = m.cfg
    # make LoRA non-trivial so the adapters are exercised, then fold them into HF base weights
    with torch.no_grad():
        for L in m.layers:
            for lora in (L.lora_qkv, L.lora_o, L.lora_gate_up, L.lora_down):
                for B in lora.B:
                    B.normal_(0, 0.02)
    hfc = transformers.LlamaConfig(vocab_size=c.vocab_size, hidden_size=c.hidden_size,
                                   intermediate_size=c.intermediate_size,
                                   num_hidden_layers=c.num_hidden_layers,
                                   num_attention_heads=c.num_attention_heads,
                                   num_key_value_heads=c.num_key_value_heads,
                                   max_position_embeddings=c.max_position_embeddings,
                                   rms_norm_eps=c.rms_norm_eps, rope_theta=c.rope_theta,
                                   num_labels=2, pad_token_id=0)
    hf = transformers.LlamaForSequenceClassification(hfc).eval()
    sd = dict(m.hf_state_dict())
    d, nh, nkv, I = c.head_dim, c.num_attention_heads, c.num_key_value_heads, c.intermediate_size
    r = c.lora_rank
    for i, L in enumerate(m.layers):
        p = f"model.layers.{i}."
        def fold(lora, j, rows):
            A = lora.A[j * r:(j + 1) * r]
            return (lora.B[j] @ A) * lora.scale
        sd[p + "self_attn.q_proj.weight"] = sd[p + "self_attn.q_proj.weight"] + fold(L.lora_qkv, 0, nh * d)
        sd[p + "self_attn.k_proj.weight"] = sd[p + "self_attn.k_proj.weight"] + fold(L.lora_qkv, 1, nkv * d)
        sd[p + "self_attn.v_proj.weight"] = sd[p + "self_attn.v_proj.weight"] + fold(L.lora_qkv, 2, nkv * d)
        sd[p + "self_attn.o_proj.weight"] = sd[p + "self_attn.o_proj.weight"] + fold(L.lora_o, 0, None)
        sd[p + "mlp.gate_proj.weight"] = sd[p + "mlp.gate_proj.weight"] + fold(L.lora_gate_up, 0, I)
        sd[p + "mlp.up_proj.weight"] = sd[p + "mlp.up_proj.weight"] + fold(L.lora_gate_up, 1, I)
        sd[p + "mlp.down_proj.weight"] = sd[p + "mlp.down_proj.weight"] + fold(L.lora_down, 0, None)
    hf.load_state_dict(sd, strict=True)
    b = _batch(c.vocab_size, 128, 4)
    with torch.no_grad():
        ours = m.forward_padded(b.input_ids, b.attention_mask)
        # HF picks the last non-pad token; right padding with pad id 0 -> same rows
        ref = hf(input_ids=b.input_ids, attention_mask=b.attention_mask).logits
    torch.testing.assert_close(ours, ref, atol=1e-4, rtol=1e-3)


@pytest.mark.parametrize("name", ["tiny-bert", "tiny-albert", "tiny-distilbert", "tiny-llama-lora"])
def test_filler_row_padding_is_invisible(name):
    from bcfl.data.batching import make_packed_batch, pad_packed
    m = build_model(name, num_labels=2, seed=0, dtype=torch.float32).eval()
    ds = load_split("tiny", "train", m.cfg.vocab_size, 128)
    b = make_packed_batch(ds, np.arange(0, 70, 7))
    pb = pad_packed(b, 64)
    assert pb.num_tokens % 64 == 0 and pb.num_tokens > b.num_tokens and pb.batch_size == b.batch_size
    with torch.no_grad():
        torch.testing.assert_close(m(pb), m(b), atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("name,labels,count,params", [
    ("biobert", 41, 201, 108_341_801),
    ("albert-base-v2", 2, 27, 11_685_122),
    ("distilbert", 2, 104, 66_955_010),
])
def test_reference_state_dict_layouts(name, labels, count, params):
    m = build_model(name, num_labels=labels, device="meta")
    sd = m.hf_state_dict()
    assert len(sd) == count
    assert sum(t.numel() for t in sd.values()) == params


def test_llama8b_lora_trainable_size():
    m = build_model("llama3-8b-lora", num_labels=2, device="meta", dtype=torch.bfloat16)
    n = sum(p.numel() for p in m.parameters() if p.requires_grad)
    assert 41_900_000 < n < 42_000_000  # 41.94 M LoRA + 8192 score
    assert len(m.adapter_items()) == 32 * 14 + 1


@pytest.mark.parametrize("name", ["tiny-bert", "tiny-albert", "tiny-distilbert", "tiny-llama-lora"])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_pooled_rows_only_last_layer_is_exact(name, p):
    """The last layer computing only the pooled rows gives the same logits and the same gradient
    for every parameter as the full last layer (incl. attention-dropout masks)."""
    from bcfl.ops import rng as _rng
    from bcfl.data.batching import make_packed_batch
    from bcfl.data.registry import load_split
    m = build_model(name, num_labels=3, seed=0, dtype=torch.float32)
    for mod in m.modules():  # attention-probability dropout only: hidden dropout hashes row ids
        for attr in ("attention_probs_dropout_prob", "attention_dropout"):
            if hasattr(getattr(mod, "cfg", None), attr):
                setattr(mod.cfg, attr, p)
        for attr in ("hidden_dropout_prob", "dropout", "classifier_dropout_prob", "seq_classif_dropout"):
            if hasattr(getattr(mod, "cfg", None), attr):
                setattr(mod.cfg, attr, 0.0)
    ds = load_split("tiny", "train", 2048, 128)
    b = make_packed_batch(ds, np.arange(0, 300, 23))
    out = {}
    for flag in (False, True):
        m.pooled_rows_only = flag
        m.train()
        _rng.manual_seed(11)
        for q in m.parameters():
            q.grad = None
        logits = m(b)
        logits.float().pow(2).sum().backward()
        out[flag] = (logits.detach().clone(), [q.grad.clone() for q in m.parameters() if q.grad is not None])
    torch.testing.assert_close(out[True][0], out[False][0], atol=1e-5, rtol=1e-4)
    assert len(out[True][1]) == len(out[False][1])
    for a, c in zip(out[True][1], out[False][1]):
        torch.testing.assert_close(a, c, atol=1e-5, rtol=1e-4)
