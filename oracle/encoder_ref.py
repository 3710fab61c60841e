"""fp32 CPU restatement of the BERT / XLM-R encoders (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

The reference sends text to remote servers running BAAI/bge-* (embedding, litellm.embedding at
super_rag/llm/embed/embedding_service.py:168-175) and BAAI/bge-reranker-* (cross-encoder,
litellm.arerank at super_rag/llm/rerank/rerank_service.py:95-104).  Those models are public
architectures outside the reference:
  * BERT (bge-small/base/large-en): post-LN encoder, absolute positions 0..S-1, token types.
  * XLM-R (bge-m3, bge-reranker-*): same block, positions padding_idx + cumsum(ids != pad),
    classification head dense -> tanh -> out_proj on the first token.
  * Sentence embedding = CLS pooling (BGE model cards) or masked mean, then L2 normalisation.
This module is pinned to ``transformers`` on identical weights in tests/test_oracle.py.
Weights use Hugging Face names without the model prefix ("embeddings.word_embeddings.weight", ...).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch


@dataclass
class RefConfig:
    vocab_size: int
    hidden: int
    layers: int
    heads: int
    intermediate: int
    max_position: int
    type_vocab: int
    ln_eps: float
    position_offset: int = 0      # XLM-R: padding_idx (1); BERT: 0
    classifier: int = 0
    num_labels: int = 1


def position_ids(ids: torch.Tensor, offset: int) -> torch.Tensor:
    if offset == 0:
        return torch.arange(ids.shape[1], device=ids.device).unsqueeze(0).expand_as(ids)
    m = (ids != offset).long()
    return torch.cumsum(m, dim=1) * m + offset


def _ln(x, w, b, eps):
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), w, b, eps)


def _t(w, name):
    v = w[name]
    return v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v), dtype=torch.float32)


@torch.no_grad()
def e4m3(x: torch.Tensor) -> torch.Tensor:
    """OCP e4m3fn rounding (nearest even, saturating at +-448) back to fp32."""
    return x.clamp(-448.0, 448.0).to(torch.float8_e4m3fn).to(torch.float32)


def fp8_rows(wt: torch.Tensor) -> torch.Tensor:
    """The fp8 FFN mode's weight copy: per row the largest power of two 2^e with
    max|w| 2^e <= 448, e4m3(w 2^e) 2^-e (the device quantises the fp16 weight)."""
    amax = wt.abs().amax(1, keepdim=True)
    e = torch.floor(torch.log2(448.0 / amax.clamp_min(1e-30)))
    e = torch.where(amax * torch.exp2(e + 1) <= 448.0, e + 1, e)
    e = torch.where(amax * torch.exp2(e) > 448.0, e - 1, e)
    return e4m3(wt * torch.exp2(e)) * torch.exp2(-e)


def _fold8(u, g, beta, wt, bias, eps):
    """fp8 mode 2's LayerNorm-folded GEMM LN(u) W^T + b on e4m3 operands: the device keeps the
    pre-LN residual sum u (fp16) and its row statistics, multiplies e4m3(u) by the e4m3 row copy
    of the folded weight W' = fp16(W diag(gamma)) and undoes the normalisation in the epilogue:
    rstd (e4m3(u) W'^T - mu colsum(W')) + (W beta + b)  (super-rag_amd/csrc/encoder.cpp fp8_ >= 2)."""
    mu = u.mean(-1, keepdim=True)
    rstd = torch.rsqrt(((u - mu) ** 2).mean(-1, keepdim=True) + eps)
    wq = fp8_rows((wt * g[None, :]).half().float())
    return rstd * (e4m3(u.half().float()) @ wq.T - mu * wq.sum(1)) + (wt @ beta + bias)


def encode_hidden(cfg: RefConfig, w: dict, ids, mask, type_ids=None,
                  fp8_ffn: bool = False, fp8: int = 0) -> torch.Tensor:
    """Final hidden states [B, S, d] in fp32.  fp8 (the library's opt-in precision modes;
    fp8_ffn=True is fp8=1): 1 = the FFN activations 2 GELU(.) rounded to e4m3 and multiplied by
    fp8_rows(fp16(W2 / 2)); 2 = also FFN1 and the QKV of layers >= 1 as _fold8 on the pre-LN
    residual sums; 3 = FFN1 as in 2, QKV in fp16 (super-rag_amd/csrc/encoder.cpp ffn1_8 / qkv_8)."""
    fp8 = max(fp8, 1 if fp8_ffn else 0)
    # weights given as torch tensors on a device (e.g. fp32 on the GPU for the long-sequence
    # checks) run the same restatement there; numpy weights run on the CPU
    dev = _t(w, "embeddings.word_embeddings.weight").device
    ids = torch.as_tensor(np.asarray(ids), dtype=torch.long, device=dev)
    mask = torch.as_tensor(np.asarray(mask), dtype=torch.float32, device=dev)
    B, S = ids.shape
    tt = torch.zeros_like(ids) if type_ids is None else \
        torch.as_tensor(np.asarray(type_ids), dtype=torch.long, device=dev)
    pos = position_ids(ids, cfg.position_offset)
    x = (_t(w, "embeddings.word_embeddings.weight")[ids]
         + _t(w, "embeddings.position_embeddings.weight")[pos]
         + _t(w, "embeddings.token_type_embeddings.weight")[tt])
    h = _ln(x, _t(w, "embeddings.LayerNorm.weight"), _t(w, "embeddings.LayerNorm.bias"), cfg.ln_eps)
    d, H = cfg.hidden, cfg.heads
    dh = d // H
    bias = (1.0 - mask)[:, None, None, :] * torch.finfo(torch.float32).min
    for l in range(cfg.layers):
        p = f"encoder.layer.{l}."
        def lin(x, n):
            return x @ _t(w, p + n + ".weight").T + _t(w, p + n + ".bias")
        if fp8 == 2 and l > 0:
            pp = f"encoder.layer.{l - 1}.output.LayerNorm."
            wqkv = torch.cat([_t(w, p + f"attention.self.{n}.weight") for n in ("query", "key", "value")])
            bqkv = torch.cat([_t(w, p + f"attention.self.{n}.bias") for n in ("query", "key", "value")])
            q, k, v = _fold8(u2, _t(w, pp + "weight"), _t(w, pp + "bias"), wqkv, bqkv,
                             cfg.ln_eps).split(d, dim=-1)
        else:
            q, k, v = lin(h, "attention.self.query"), lin(h, "attention.self.key"), lin(h, "attention.self.value")
        q = q.reshape(B, S, H, dh).transpose(1, 2)
        k = k.reshape(B, S, H, dh).transpose(1, 2)
        v = v.reshape(B, S, H, dh).transpose(1, 2)
        s = q @ k.transpose(-1, -2) / math.sqrt(dh) + bias
        ctx = (s.softmax(-1) @ v).transpose(1, 2).reshape(B, S, d)
        u1 = lin(ctx, "attention.output.dense") + h
        g1, b1 = _t(w, p + "attention.output.LayerNorm.weight"), _t(w, p + "attention.output.LayerNorm.bias")
        h = _ln(u1, g1, b1, cfg.ln_eps)
        if fp8 >= 2:
            f = torch.nn.functional.gelu(_fold8(u1, g1, b1, _t(w, p + "intermediate.dense.weight"),
                                                _t(w, p + "intermediate.dense.bias"), cfg.ln_eps))
        else:
            f = torch.nn.functional.gelu(lin(h, "intermediate.dense"))
        if fp8:
            w2 = fp8_rows((0.5 * _t(w, p + "output.dense.weight")).half().float())
            o = e4m3(2.0 * f) @ w2.T + _t(w, p + "output.dense.bias")
        else:
            o = lin(f, "output.dense")
        u2 = o + h
        h = _ln(u2, _t(w, p + "output.LayerNorm.weight"), _t(w, p + "output.LayerNorm.bias"), cfg.ln_eps)
    return h


@torch.no_grad()
def embed(cfg: RefConfig, w: dict, ids, mask, type_ids=None, pool: str = "cls") -> np.ndarray:
    """Sentence embeddings [B, d], pooled then L2-normalised (fp32)."""
    h = encode_hidden(cfg, w, ids, mask, type_ids)
    m = torch.as_tensor(np.asarray(mask), dtype=torch.float32, device=h.device)
    if pool == "cls":
        e = h[:, 0]
    else:
        e = (h * m[..., None]).sum(1) / m.sum(1, keepdim=True).clamp_min(1e-30)
    n = e.norm(dim=-1, keepdim=True)
    e = torch.where(n > 0, e / n, torch.zeros_like(e))
    return e.cpu().numpy()


@torch.no_grad()
def cross_logits(cfg: RefConfig, w: dict, ids, mask, type_ids=None, fp8_ffn: bool = False,
                 fp8: int = 0) -> np.ndarray:
    """RoBERTa classification head on the first token: [P, num_labels] raw logits."""
    h = encode_hidden(cfg, w, ids, mask, type_ids, fp8_ffn, fp8)[:, 0]
    t = torch.tanh(h @ _t(w, "classifier.dense.weight").T + _t(w, "classifier.dense.bias"))
    return (t @ _t(w, "classifier.out_proj.weight").T + _t(w, "classifier.out_proj.bias")).cpu().numpy()


def longest_first(a: int, b: int, budget: int):
    """Lengths kept by Hugging Face fast tokenizers' LongestFirst pair truncation
    (tokenizers utils/truncation.rs): the shorter side is kept whole when it fits in half the
    budget, otherwise both are cut to half and the longer side (the second on ties) gets the odd
    token.  bge rerankers load the fast tokenizer and call tokenizer(pairs, truncation=True)."""
    budget = max(budget, 0)
    if a + b <= budget:
        return a, b
    swap = a > b
    n1, n2 = (b, a) if swap else (a, b)
    n2 = n1 if n1 > budget else max(n1, budget - n1)
    if n1 + n2 > budget:
        n1 = budget // 2
        n2 = n1 + budget % 2
    if swap:
        n1, n2 = n2, n1
    return min(a, n1), min(b, n2)


def pack_pairs(q_tok, q_len, p_tok, p_len, rows, S, style, bos, eos, pad):
    """Reference packing of (query, passage) pairs — HF tokenizer pair layout with 'longest_first'
    truncation (see longest_first).
    style 0: <s> q </s></s> p </s>;  style 1: [CLS] q [SEP] p [SEP] (token type 1 on the passage)."""
    B, K = rows.shape
    ids = np.full((B * K, S), pad, dtype=np.int32)
    msk = np.zeros((B * K, S), dtype=np.int32)
    typ = np.zeros((B * K, S), dtype=np.int32)
    nspec = 4 if style == 0 else 3
    for b in range(B):
        for j in range(K):
            r = int(rows[b, j])
            q = list(q_tok[b][: q_len[b]])
            p = list(p_tok[r][: p_len[r]]) if r >= 0 else []
            lq2, lp2 = longest_first(len(q), len(p), S - nspec)
            q, p = q[:lq2], p[:lp2]
            if style == 0:
                seq = [bos] + q + [eos, eos] + p + [eos]
                tps = [0] * len(seq)
            else:
                seq = [bos] + q + [eos] + p + [eos]
                tps = [0] * (len(q) + 2) + [1] * (len(p) + 1)
            i = b * K + j
            ids[i, : len(seq)] = seq
            msk[i, : len(seq)] = 1
            typ[i, : len(seq)] = tps
    return ids, msk, typ
