"""Encoder models (BGE embedders and cross-encoder rerankers) on the MI355X library.

Model shapes follow the public model cards of the models the reference calls remotely
(super_rag/migration/sql/model_configs_init.sql seeds BAAI/bge-m3 for embedding and
BAAI/bge-reranker-v2-m3 for rerank).  Weights come from a Hugging Face model directory
``$SUPER_RAG_AMD_WEIGHTS/<model>/`` (``model.safetensors``; a ``config.json`` there also defines
models not in MODELS) or an explicit ``checkpoint=`` path.  A missing checkpoint is an error:
seeded random weights of identical shape (benchmarks, tests) need the explicit opt-in
``SUPER_RAG_AMD_SYNTHETIC=1`` or ``weights=random_weights(...)``, so a misconfigured deployment
cannot serve meaningless embeddings silently.
"""
from __future__ import annotations

import ctypes
import json
import logging
import os
from dataclasses import dataclass, field, replace

import numpy as np

from . import _native as N

logger = logging.getLogger(__name__)


class ModelAssetsError(FileNotFoundError):
    """A model's checkpoint / config / tokenizer is missing or unusable."""


def synthetic_allowed() -> bool:
    """Explicit opt-in for seeded random weights and the hashing tokenizer (tests, benchmarks)."""
    return os.environ.get("SUPER_RAG_AMD_SYNTHETIC", "") not in ("", "0", "false", "False")


def weights_root() -> str | None:
    return os.environ.get("SUPER_RAG_AMD_WEIGHTS") or None


def model_dir(name: str) -> str | None:
    """$SUPER_RAG_AMD_WEIGHTS/<name> (the org prefix of "BAAI/bge-m3" is dropped), if set."""
    root = weights_root()
    return os.path.join(root, name.split("/")[-1]) if root else None


@dataclass(frozen=True)
class ModelSpec:
    name: str
    arch: str                # "bert" | "xlmr"
    vocab_size: int
    hidden: int
    layers: int
    heads: int
    intermediate: int
    max_position: int
    type_vocab: int
    ln_eps: float
    position_offset: int     # XLM-R padding_idx, 0 for BERT
    pool: str = "cls"        # sentence embedding pooling (BGE: CLS)
    classifier: int = 0      # 1: RoBERTa classification head (rerankers)
    num_labels: int = 1
    # special tokens (BERT: [CLS]=101 [SEP]=102 [PAD]=0; XLM-R: <s>=0 </s>=2 <pad>=1)
    bos_id: int = 101
    eos_id: int = 102
    pad_id: int = 0
    max_length: int = 512
    residual_fp16: bool = False  # fp16 residual stream (rerankers: ranking fidelity, less traffic)
    # the model directory the spec was resolved from (its checkpoint and tokenizer live there);
    # None: $SUPER_RAG_AMD_WEIGHTS/<name>
    source_dir: str | None = field(default=None, compare=False)

    @property
    def pair_style(self) -> int:
        return 0 if self.arch == "xlmr" else 1

    @property
    def asset_dir(self) -> str | None:
        """Directory holding model.safetensors / tokenizer.json for this spec, or None."""
        return self.source_dir or model_dir(self.name)


def _bert(name, d, L, H, F, **kw):
    return ModelSpec(name, "bert", 30522, d, L, H, F, 512, 2, 1e-12, 0, **kw)


def _xlmr(name, d, L, H, F, max_pos=514, **kw):
    return ModelSpec(name, "xlmr", 250002, d, L, H, F, max_pos, 1, 1e-5, 1, bos_id=0, eos_id=2,
                     pad_id=1, max_length=max_pos - 2, **kw)


MODELS = {
    "bge-small-en": _bert("bge-small-en", 384, 12, 12, 1536),
    "bge-base-en": _bert("bge-base-en", 768, 12, 12, 3072),
    "bge-large-en": _bert("bge-large-en", 1024, 24, 16, 4096),
    "bge-m3": _xlmr("bge-m3", 1024, 24, 16, 4096, max_pos=8194),
    "bge-reranker-base": _xlmr("bge-reranker-base", 768, 12, 12, 3072, classifier=1,
                               residual_fp16=True),
    "bge-reranker-large": _xlmr("bge-reranker-large", 1024, 24, 16, 4096, classifier=1,
                                residual_fp16=True),
    "bge-reranker-v2-m3": _xlmr("bge-reranker-v2-m3", 1024, 24, 16, 4096, max_pos=8194,
                                classifier=1, residual_fp16=True),
}


def _key(model: str) -> str:
    key = model.split("/")[-1].lower()
    for suffix in ("-v1.5", "-v1"):
        if key.endswith(suffix):
            key = key[: -len(suffix)]
    return key


def spec_from_dir(path: str, name: str | None = None) -> ModelSpec:
    """ModelSpec of a Hugging Face BERT / XLM-R model directory: config.json (shapes, head),
    tokenizer.json (special-token ids), 1_Pooling/config.json (sentence-transformers pooling)."""
    cfg_path = os.path.join(path, "config.json")
    try:
        with open(cfg_path, encoding="utf-8") as f:
            cfg = json.load(f)
    except OSError as e:
        raise ModelAssetsError(f"model config not found: {cfg_path}") from e
    mt = cfg.get("model_type", "")
    if mt == "bert":
        arch = "bert"
    elif mt in ("xlm-roberta", "roberta"):
        arch = "xlmr"
    else:
        raise ModelAssetsError(f"{cfg_path}: unsupported model_type '{mt}' (bert, xlm-roberta)")
    if cfg.get("hidden_act", "gelu") != "gelu":
        raise ModelAssetsError(f"{cfg_path}: unsupported hidden_act '{cfg.get('hidden_act')}'")
    classifier = int(any("SequenceClassification" in a for a in cfg.get("architectures", [])))
    num_labels = max(1, len(cfg.get("id2label", {}))) if classifier else 1
    pool = "cls"
    pcfg = os.path.join(path, "1_Pooling", "config.json")
    if os.path.exists(pcfg):
        with open(pcfg, encoding="utf-8") as f:
            pc = json.load(f)
        if pc.get("pooling_mode_mean_tokens") and not pc.get("pooling_mode_cls_token"):
            pool = "mean"
    pad = int(cfg.get("pad_token_id", 0 if arch == "bert" else 1))
    if arch == "bert":
        bos, eos = 101, 102
        special = ("[CLS]", "[SEP]", "[PAD]")
    else:
        bos, eos = int(cfg.get("bos_token_id", 0)), int(cfg.get("eos_token_id", 2))
        special = ("<s>", "</s>", "<pad>")
    tok = os.path.join(path, "tokenizer.json")
    if os.path.exists(tok):
        from tokenizers import Tokenizer as HFTokenizer
        t = HFTokenizer.from_file(tok)
        ids = [t.token_to_id(s) for s in special]
        bos, eos = ids[0] if ids[0] is not None else bos, ids[1] if ids[1] is not None else eos
        pad = ids[2] if ids[2] is not None else pad
    max_pos = int(cfg["max_position_embeddings"])
    off = pad if arch == "xlmr" else 0
    return ModelSpec(name or os.path.basename(os.path.normpath(path)), arch, int(cfg["vocab_size"]),
                     int(cfg["hidden_size"]), int(cfg["num_hidden_layers"]),
                     int(cfg["num_attention_heads"]), int(cfg["intermediate_size"]), max_pos,
                     int(cfg.get("type_vocab_size", 2 if arch == "bert" else 1)),
                     float(cfg.get("layer_norm_eps", 1e-12 if arch == "bert" else 1e-5)), off,
                     pool=pool, classifier=classifier, num_labels=num_labels, bos_id=bos,
                     eos_id=eos, pad_id=pad, max_length=max_pos - off - (1 if off else 0),
                     residual_fp16=bool(classifier))


def resolve_spec(model: str) -> ModelSpec:
    """Map a reference model name (e.g. "BAAI/bge-m3", "bge-base-en-v1.5") to a ModelSpec: the
    built-in shapes of MODELS, else the config.json of $SUPER_RAG_AMD_WEIGHTS/<model>.  The
    directory is looked up under the name as given (its case and version suffix kept, as Hugging
    Face names it: ".../bge-base-en-v1.5"), and the spec remembers it, so the checkpoint and the
    tokenizer come from the same directory the spec did."""
    key = _key(model)
    d = model_dir(model)
    has_dir = bool(d) and os.path.isdir(d)
    if key in MODELS:
        return replace(MODELS[key], source_dir=d) if has_dir else MODELS[key]
    if has_dir and os.path.exists(os.path.join(d, "config.json")):
        return replace(spec_from_dir(d, key), source_dir=d)
    raise KeyError(f"unknown encoder model '{model}' (known: {sorted(MODELS)}; or a model "
                   f"directory with config.json under SUPER_RAG_AMD_WEIGHTS)")


def weight_shapes(spec: ModelSpec) -> dict:
    d, F = spec.hidden, spec.intermediate
    s = {
        "embeddings.word_embeddings.weight": (spec.vocab_size, d),
        "embeddings.position_embeddings.weight": (spec.max_position, d),
        "embeddings.token_type_embeddings.weight": (spec.type_vocab, d),
        "embeddings.LayerNorm.weight": (d,),
        "embeddings.LayerNorm.bias": (d,),
    }
    for l in range(spec.layers):
        p = f"encoder.layer.{l}."
        for n in ("query", "key", "value"):
            s[p + f"attention.self.{n}.weight"] = (d, d)
            s[p + f"attention.self.{n}.bias"] = (d,)
        s[p + "attention.output.dense.weight"] = (d, d)
        s[p + "attention.output.dense.bias"] = (d,)
        s[p + "attention.output.LayerNorm.weight"] = (d,)
        s[p + "attention.output.LayerNorm.bias"] = (d,)
        s[p + "intermediate.dense.weight"] = (F, d)
        s[p + "intermediate.dense.bias"] = (F,)
        s[p + "output.dense.weight"] = (d, F)
        s[p + "output.dense.bias"] = (d,)
        s[p + "output.LayerNorm.weight"] = (d,)
        s[p + "output.LayerNorm.bias"] = (d,)
    if spec.classifier:
        s["classifier.dense.weight"] = (d, d)
        s["classifier.dense.bias"] = (d,)
        s["classifier.out_proj.weight"] = (spec.num_labels, d)
        s["classifier.out_proj.bias"] = (spec.num_labels,)
    return s


def random_weights(spec: ModelSpec, seed: int = 0, style: str = "test") -> dict:
    """Seeded synthetic weights of the model's exact shapes.

    style="hf":   BERT initialisation (N(0, 0.02) matrices/embeddings, LN = (1, 0), biases 0).
    style="test": additionally randomises biases and LayerNorm affine terms so every parameter
                  path is exercised by the parity tests.
    """
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in weight_shapes(spec).items():
        if name.endswith("LayerNorm.weight"):
            v = np.ones(shape, np.float32)
            if style == "test":
                v += 0.1 * rng.standard_normal(shape, dtype=np.float32)
        elif name.endswith("LayerNorm.bias") or name.endswith(".bias"):
            v = (0.02 * rng.standard_normal(shape, dtype=np.float32) if style == "test"
                 else np.zeros(shape, np.float32))
        else:
            v = 0.02 * rng.standard_normal(shape, dtype=np.float32)
        out[name] = v
    if spec.arch == "xlmr":
        out["embeddings.position_embeddings.weight"][spec.position_offset] = 0.0  # padding_idx row
    return out


_PREFIXES = ("bert.", "roberta.", "model.", "xlm_roberta.")


def canonical_name(name: str) -> str:
    for p in _PREFIXES:
        if name.startswith(p):
            name = name[len(p):]
    return name.replace("LayerNorm.gamma", "LayerNorm.weight").replace("LayerNorm.beta", "LayerNorm.bias")


def load_safetensors(path: str) -> dict:
    from safetensors.numpy import load_file
    return {canonical_name(k): v.astype(np.float32) for k, v in load_file(path).items()}


def find_checkpoint(spec: ModelSpec) -> str | None:
    """$SUPER_RAG_AMD_WEIGHTS/<model>/model.safetensors, or None when the variable is unset.
    Raises ModelAssetsError when the variable is set but the file is missing (misconfiguration)."""
    d = spec.asset_dir
    if d is None:
        return None
    p = os.path.join(d, "model.safetensors")
    if not os.path.exists(p):
        raise ModelAssetsError(f"checkpoint for {spec.name} not found: {p}")
    return p


def model_weights(spec: ModelSpec, checkpoint: str | None = None, seed: int = 0,
                  init_style: str = "hf") -> dict:
    """The weights an Encoder loads when none are passed: the explicit or configured
    checkpoint, else seeded random weights under the explicit synthetic opt-in, else an error."""
    ckpt = checkpoint or find_checkpoint(spec)
    if ckpt:
        if not os.path.exists(ckpt):
            raise ModelAssetsError(f"checkpoint for {spec.name} not found: {ckpt}")
        return load_safetensors(ckpt)
    if synthetic_allowed():
        logger.warning("%s: no checkpoint, using seeded random weights (SUPER_RAG_AMD_SYNTHETIC)",
                       spec.name)
        return random_weights(spec, seed, init_style)
    raise ModelAssetsError(
        f"no weights for {spec.name}: set SUPER_RAG_AMD_WEIGHTS to a directory holding "
        f"{spec.name}/model.safetensors (or pass checkpoint=); seeded random weights need the "
        f"explicit opt-in SUPER_RAG_AMD_SYNTHETIC=1")


class Encoder:
    """One encoder instance resident on one device (sr_encoder_* in the C-ABI)."""

    def __init__(self, spec: ModelSpec, device: int = 0, weights: dict | None = None,
                 seed: int = 0, max_tokens: int = 0, init_style: str = "hf",
                 checkpoint: str | None = None):
        if weights is None:   # resolve first: a missing checkpoint fails before any device work
            weights = model_weights(spec, checkpoint, seed, init_style)
        N.require_gpu()
        self.spec = spec
        self.device = int(device)
        cfg = N.EncoderConfigC(spec.vocab_size, spec.hidden, spec.layers, spec.heads,
                               spec.intermediate, spec.max_position, spec.type_vocab,
                               float(spec.ln_eps), spec.position_offset, spec.classifier,
                               spec.num_labels, int(max_tokens), int(spec.residual_fp16))
        h = ctypes.c_void_p()
        N.call("sr_encoder_create", ctypes.byref(cfg), self.device, ctypes.byref(h))
        self._h = h
        self.load_weights(weights)

    def load_weights(self, weights: dict) -> None:
        for name, v in weights.items():
            name = canonical_name(name)
            if name.endswith("position_ids") or name.startswith("pooler."):
                continue
            a = np.ascontiguousarray(np.asarray(v, dtype=np.float32))
            N.call("sr_encoder_set_weight", self._h, name.encode(), N.ptr(a), a.size)
        N.call("sr_encoder_ready", self._h)

    def set_fp8(self, mode: int) -> None:
        """Opt-in fp8 precision mode (LN-folded fp16-residual encoders, e.g. cross-encoders):
        1 = FFN2 on the block-scaled fp8 MFMA (e4m3 FFN activations), 2 = also FFN1 and the QKV
        of layers >= 1 on e4m3 copies of the residual sums (faster, ranks worse), 3 = FFN1 and
        FFN2 as in 2 with QKV + attention in fp16 (fused), 0 = fp16 (sr_encoder_set_fp8).  Modes
        4 (QKV on normalised e4m3 rows) and 5 (mode 3 + the O-projection on e4m3 attention
        outputs) failed the ranking fidelity gates: diagnostic library only."""
        N.call("sr_encoder_set_fp8", self._h, int(mode))

    def set_fp8_ffn(self, on: bool = True) -> None:
        self.set_fp8(1 if on else 0)

    def close(self) -> None:
        if getattr(self, "_h", None):
            N.load().sr_encoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- host API ---------------------------------------------------------------------------------
    def embed(self, ids, mask, type_ids=None, pool: str | None = None) -> np.ndarray:
        ids = np.ascontiguousarray(np.asarray(ids, dtype=np.int32))
        mask = np.ascontiguousarray(np.asarray(mask, dtype=np.int32))
        tt = None if type_ids is None else np.ascontiguousarray(np.asarray(type_ids, dtype=np.int32))
        B, S = ids.shape
        out = np.empty((B, self.spec.hidden), dtype=np.float32)
        p = N.SR_POOL_CLS if (pool or self.spec.pool) == "cls" else N.SR_POOL_MEAN
        N.call("sr_encoder_forward", self._h, N.ptr(ids), N.ptr(mask), N.ptr(tt), B, S, p,
               N.ptr(out))
        return out

    def cross_score(self, ids, mask, type_ids=None) -> np.ndarray:
        ids = np.ascontiguousarray(np.asarray(ids, dtype=np.int32))
        mask = np.ascontiguousarray(np.asarray(mask, dtype=np.int32))
        tt = None if type_ids is None else np.ascontiguousarray(np.asarray(type_ids, dtype=np.int32))
        P, S = ids.shape
        out = np.empty((P, self.spec.num_labels), dtype=np.float32)
        N.call("sr_cross_score", self._h, N.ptr(ids), N.ptr(mask), N.ptr(tt), P, S, N.ptr(out))
        return out

    # -- device API -------------------------------------------------------------------------------
    def embed_dev(self, ids, mask, type_ids=None, out=None, ld_out: int | None = None,
                  fp16: bool = True, pool: str | None = None, stream=None):
        import torch
        B, S = ids.shape
        ld = ld_out or self.spec.hidden
        if out is None:
            out = torch.empty((B, ld), dtype=torch.float16 if fp16 else torch.float32,
                              device=ids.device)
        dt = N.SR_DTYPE_F16 if out.dtype == torch.float16 else N.SR_DTYPE_F32
        p = N.SR_POOL_CLS if (pool or self.spec.pool) == "cls" else N.SR_POOL_MEAN
        N.call("sr_encoder_forward_dev", self._h, N.ptr(ids), N.ptr(mask), N.ptr(type_ids), B, S,
               p, N.ptr(out), dt, out.shape[1], N.stream_handle(stream))
        return out

    def cross_score_dev(self, ids, mask, type_ids=None, out=None, stream=None):
        import torch
        P, S = ids.shape
        if out is None:
            out = torch.empty((P, self.spec.num_labels), dtype=torch.float32, device=ids.device)
        N.call("sr_cross_score_dev", self._h, N.ptr(ids), N.ptr(mask), N.ptr(type_ids), P, S,
               N.ptr(out), N.stream_handle(stream))
        return out


def build_pairs_dev(q_tok, q_len, p_tok, p_len, cand_rows, S: int, spec: ModelSpec, with_types=False,
                    stream=None):
    """Pack (query, candidate passage) token pairs on the device (sr_build_pairs_dev)."""
    import torch
    B, K = cand_rows.shape
    dev = cand_rows.device
    ids = torch.empty((B * K, S), dtype=torch.int32, device=dev)
    mask = torch.empty((B * K, S), dtype=torch.int32, device=dev)
    types = torch.empty((B * K, S), dtype=torch.int32, device=dev) if with_types else None
    N.call("sr_build_pairs_dev", N.ptr(q_tok), N.ptr(q_len), q_tok.shape[1], N.ptr(p_tok),
           N.ptr(p_len), p_tok.shape[1], N.ptr(cand_rows), B, K, S, spec.pair_style, spec.bos_id,
           spec.eos_id, spec.pad_id, N.ptr(ids), N.ptr(mask), N.ptr(types), dev.index or 0,
           N.stream_handle(stream))
    return ids, mask, types


def rerank_select_dev(logits, k_out: int, stream=None):
    """[B, K] fp32 logits -> [B, k_out] int32 candidate positions (logit desc, position asc)."""
    import torch
    B, K = logits.shape
    out = torch.empty((B, k_out), dtype=torch.int32, device=logits.device)
    N.call("sr_rerank_select_dev", N.ptr(logits), B, K, int(k_out), N.ptr(out),
           logits.device.index or 0, N.stream_handle(stream))
    return out
