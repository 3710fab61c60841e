"""Test helper: write small Hugging Face model directories offline (config.json, model.safetensors,
tokenizer.json, optional 1_Pooling/config.json) — the layout a deployment points
SUPER_RAG_AMD_WEIGHTS at.  Weights are seeded random (no checkpoints offline); the vocabularies are
real `tokenizers` models (BERT WordPiece, XLM-R-style Unigram) over a small word list.
"""
from __future__ import annotations

import json
import os

import numpy as np

WORDS = ("the a an of to in and or is are was were be for on with by at from as that this it "
         "data vector search query rank score model gpu memory kernel index store text chunk "
         "document passage answer question embedding cosine distance matrix tile wave lane cache "
         "fast slow small large first last new old good best top result user system node flow "
         "merge rerank filter collection token batch stream layer head attention norm sum mean "
         "apple banana cherry grape lemon mango orange peach pear plum river mountain forest ocean "
         "city road bridge tower castle garden music paper pencil window door table chair light "
         "sound color water fire earth wind stone metal glass wood cloud rain snow storm sun moon "
         "star planet rocket engine wheel motor signal network packet server client request").split()


def bert_tokenizer_json(path: str) -> dict:
    """BERT-style WordPiece tokenizer: [PAD]=0 [UNK]=1 [CLS]=2 [SEP]=3, words, ##suffixes."""
    from tokenizers import Tokenizer, decoders, models, normalizers, pre_tokenizers, processors
    vocab = {t: i for i, t in enumerate(["[PAD]", "[UNK]", "[CLS]", "[SEP]"] + list(WORDS)
                                        + ["##s", "##ing", "##ed", "##er"])}
    tk = Tokenizer(models.WordPiece(vocab, unk_token="[UNK]"))
    tk.normalizer = normalizers.BertNormalizer(lowercase=True)
    tk.pre_tokenizer = pre_tokenizers.BertPreTokenizer()
    tk.decoder = decoders.WordPiece()
    tk.post_processor = processors.TemplateProcessing(
        single="[CLS] $A [SEP]", pair="[CLS] $A [SEP] $B:1 [SEP]:1",
        special_tokens=[("[CLS]", 2), ("[SEP]", 3)])
    tk.save(path)
    return vocab


def xlmr_tokenizer_json(path: str) -> dict:
    """XLM-R-style Unigram tokenizer: <s>=0 <pad>=1 </s>=2 <unk>=3, '▁word' pieces + chars."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, processors
    pieces = [("<s>", 0.0), ("<pad>", 0.0), ("</s>", 0.0), ("<unk>", 0.0)]
    pieces += [("▁" + w, -3.0 - 0.01 * i) for i, w in enumerate(WORDS)]
    pieces += [(c, -8.0) for c in "abcdefghijklmnopqrstuvwxyz"] + [("▁", -5.0)]
    tk = Tokenizer(models.Unigram(pieces, unk_id=3))
    tk.pre_tokenizer = pre_tokenizers.Metaspace()
    tk.decoder = decoders.Metaspace()
    tk.post_processor = processors.RobertaProcessing(("</s>", 2), ("<s>", 0))
    tk.save(path)
    return {p: i for i, (p, _) in enumerate(pieces)}


def write_model_dir(root: str, name: str, arch: str, hidden=128, layers=2, heads=2, inter=256,
                    max_pos=130, classifier=False, seed=0, pool="cls", vocab_size=None,
                    write_tokenizer=True, write_weights=True, head_scale=1.0) -> str:
    """Write root/name/{config.json, model.safetensors, tokenizer.json}; returns the directory.
    The checkpoint uses the transformers key prefixes (bert. / roberta.) of real BGE files."""
    from safetensors.numpy import save_file

    from super_rag_amd.encoder import ModelSpec, random_weights
    d = os.path.join(root, name)
    os.makedirs(d, exist_ok=True)
    tok_path = os.path.join(d, "tokenizer.json")
    vocab = (bert_tokenizer_json if arch == "bert" else xlmr_tokenizer_json)(tok_path)
    if not write_tokenizer:
        os.remove(tok_path)
    V = vocab_size or len(vocab) + 8
    if arch == "bert":
        cfg = {"model_type": "bert", "architectures": ["BertModel"], "vocab_size": V,
               "hidden_size": hidden, "num_hidden_layers": layers, "num_attention_heads": heads,
               "intermediate_size": inter, "max_position_embeddings": max_pos, "type_vocab_size": 2,
               "layer_norm_eps": 1e-12, "hidden_act": "gelu", "pad_token_id": 0}
        spec = ModelSpec(name, "bert", V, hidden, layers, heads, inter, max_pos, 2, 1e-12, 0)
        prefix = "bert."
    else:
        cfg = {"model_type": "xlm-roberta", "vocab_size": V, "hidden_size": hidden,
               "num_hidden_layers": layers, "num_attention_heads": heads, "intermediate_size": inter,
               "max_position_embeddings": max_pos, "type_vocab_size": 1, "layer_norm_eps": 1e-5,
               "hidden_act": "gelu", "pad_token_id": 1, "bos_token_id": 0, "eos_token_id": 2,
               "architectures": (["XLMRobertaForSequenceClassification"] if classifier
                                 else ["XLMRobertaModel"])}
        if classifier:
            cfg["id2label"] = {"0": "LABEL_0"}
        spec = ModelSpec(name, "xlmr", V, hidden, layers, heads, inter, max_pos, 1, 1e-5, 1,
                         classifier=int(classifier))
        prefix = "roberta."
    with open(os.path.join(d, "config.json"), "w") as f:
        json.dump(cfg, f)
    if pool == "mean":
        os.makedirs(os.path.join(d, "1_Pooling"), exist_ok=True)
        with open(os.path.join(d, "1_Pooling", "config.json"), "w") as f:
            json.dump({"pooling_mode_cls_token": False, "pooling_mode_mean_tokens": True}, f)
    w = random_weights(spec, seed, "test")
    if classifier:   # spread the logits of the random head (stable rerank order in parity tests)
        w["classifier.out_proj.weight"] *= head_scale
    if write_weights:
        save_file({(k if k.startswith("classifier.") else prefix + k): np.ascontiguousarray(v)
                   for k, v in w.items()}, os.path.join(d, "model.safetensors"))
    return d


def ref_config(spec):
    from oracle import encoder_ref as R
    return R.RefConfig(spec.vocab_size, spec.hidden, spec.layers, spec.heads, spec.intermediate,
                       spec.max_position, spec.type_vocab, spec.ln_eps, spec.position_offset,
                       spec.classifier, spec.num_labels)
