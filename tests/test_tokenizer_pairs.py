"""Pair packing: the array form of Tokenizer.encode_pairs (per-request rerank path) equals the list
form (encode_pairs_ref) and the HF LongestFirst truncation rule, on random query / passage lengths
around and beyond the budget, both pair styles (XLM-R <s> q </s></s> p </s>, BERT [CLS] q [SEP] p
[SEP] with token types), empty passages."""
import random

import numpy as np

from super_rag_amd.encoder import MODELS
from super_rag_amd.tokenizer import Tokenizer, longest_first, longest_first_arrays


def test_longest_first_arrays_equals_scalar_rule():
    bs = np.arange(0, 160)
    for a in range(0, 60, 3):
        for budget in (0, 1, 2, 3, 10, 61, 124, 125, 508):
            na, nb = longest_first_arrays(a, bs, budget)
            for b in bs:
                assert (na[b], nb[b]) == longest_first(a, int(b), budget)


def test_encode_pairs_array_form_equals_list_form():
    words = [f"w{i}" for i in range(400)]
    rng = random.Random(5)
    for name in ("bge-reranker-base", "bge-base-en"):
        tok = Tokenizer(MODELS[name], synthetic=True)
        for _ in range(120):
            q = " ".join(rng.choice(words) for _ in range(rng.randint(0, 140)))
            ps = [" ".join(rng.choice(words) for _ in range(rng.randint(0, 180)))
                  for _ in range(rng.randint(1, 24))]
            if rng.random() < 0.25:
                ps.append("")
            ml = rng.choice([None, 4, 16, 64, 128, 512])
            got, ref = tok.encode_pairs(q, ps, ml), tok.encode_pairs_ref(q, ps, ml)
            for x, y in zip(got, ref):
                assert x.dtype == y.dtype and x.shape == y.shape
                np.testing.assert_array_equal(x, y)


def test_content_cache_is_a_byte_bounded_lru():
    """one int32 array per text, bounded by bytes, hits refresh recency, results equal
    the uncached tokenisation."""
    tok = Tokenizer(MODELS["bge-reranker-base"], synthetic=True, cache_mb=0.01)  # ~10 KiB
    fresh = Tokenizer(MODELS["bge-reranker-base"], synthetic=True, cache_mb=0)
    texts = [" ".join(f"w{i}_{j}" for j in range(100)) for i in range(40)]  # ~500 B each
    for t in texts:
        assert tok.content_ids(t) == fresh.content_ids(t)
    assert tok._cache_bytes <= tok._cache_cap_bytes
    assert len(tok._cache) < len(texts)                 # evicted
    assert all(isinstance(v, np.ndarray) and v.dtype == np.int32 for v in tok._cache.values())
    assert not fresh._cache                             # cap 0: nothing kept
    hot = texts[-len(tok._cache)]                       # the oldest cached text ...
    tok.content_ids(hot)                                # ... refreshed by a hit
    for t in texts[:3]:                                 # three new entries evict the LRU ones
        tok.content_ids(t)
    assert hot in tok._cache
    many = tok.content_ids_many(texts[5:9] + texts[5:6])
    assert many == [fresh.content_ids(t) for t in texts[5:9] + texts[5:6]]


def test_content_cache_is_thread_safe_under_constant_eviction():
    # the LRU is shared by the embed worker threads, the coalescer leaders and
    # uncoalesced rerank calls; with a ~4 KiB cache every insert evicts, so an unlocked
    # get / move_to_end or pop / popitem sequence raced into KeyError and a drifting byte count
    import threading
    tok = Tokenizer(MODELS["bge-reranker-base"], synthetic=True, cache_mb=0.004)
    ref = Tokenizer(MODELS["bge-reranker-base"], synthetic=True, cache_mb=0)
    texts = [" ".join(f"t{(i * 7 + j) % 97}" for j in range(1 + i % 40)) for i in range(300)]
    want = {t: ref.content_ids(t) for t in texts}
    errors = []

    def worker(seed):
        rng = random.Random(seed)
        try:
            for _ in range(400):
                batch = [rng.choice(texts) for _ in range(rng.randint(1, 6))]
                for t, got in zip(batch, tok.content_ids_many(batch)):
                    if got != want[t]:
                        errors.append(("ids", t))
        except Exception as e:  # noqa: BLE001 - collected and asserted below
            errors.append(repr(e))

    threads = [threading.Thread(target=worker, args=(s,)) for s in range(8)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    assert not errors, errors[:3]
    held = sum(4 * int(v.size) + len(k) + 64 for k, v in tok._cache.items())
    assert tok._cache_bytes == held <= tok._cache_cap_bytes


def test_cold_rerank_requests_tokenise_off_the_event_loop():
    """a coroutine rerank request whose passages mostly miss the token cache tokenises
    in a worker thread (the HF encode would stall the loop); a warm one stays on the loop."""
    import asyncio
    import threading
    from super_rag_amd import rerank as RR
    from doubles import RelevanceEncoder, TextTokenizer

    real_tok = Tokenizer(MODELS["bge-reranker-base"], synthetic=True)
    texts = [f"passage number {i} about topic {i % 7}" for i in range(40)]
    assert real_tok.cache_misses(texts) == 40
    real_tok.encode_pairs("q", texts)
    assert real_tok.cache_misses(texts) == 0 and real_tok.cache_misses(texts + ["new"]) == 1

    tok = TextTokenizer()  # the double, with a cache that remembers what it encoded
    cached, where = set(), []
    tok.cache_misses = lambda ts: sum(t not in cached for t in ts)
    real = tok.encode_pairs

    def spy(q, ps):
        where.append(threading.current_thread() is threading.main_thread())
        cached.update(ps)
        return real(q, ps)

    tok.encode_pairs = spy
    rer = RR.RerankService("jina_ai", "r", "", "", encoder=RelevanceEncoder(tok), tokenizer=tok,
                           device_batch=256)
    cold = asyncio.run(rer._rank_texts("topic 3", texts))
    warm = asyncio.run(rer._rank_texts("topic 3", texts))
    assert cold == warm and sorted(cold) == list(range(40))
    assert where == [False, True]  # cold: a worker thread; warm: the loop (main) thread
