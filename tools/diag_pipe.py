"""Diagnostic: does the rerank stage disturb the store? (not part of the product)"""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "super-rag_amd")]
import numpy as np, torch
import bench
from super_rag_amd import _native as Nn
from super_rag_amd.encoder import MODELS, Encoder, random_weights
from super_rag_amd.store import NativeStore
from super_rag_amd.pipeline import SearchPipeline
dev = torch.device("cuda", 0)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
es, rs = MODELS["bge-base-en"], MODELS["bge-reranker-base"]
emb = Encoder(es, weights=random_weights(es, 11, "hf"), max_tokens=8192)
rer = Encoder(rs, weights=random_weights(rs, 12, "hf"), max_tokens=524288)
gc = torch.Generator(device="cpu"); gc.manual_seed(0)
centers = torch.randn((1024, 768), generator=gc).to(dev)
st = NativeStore(768, capacity=N)
for c0 in range(0, N, 1 << 20):
    st.add_dev(bench.gen_corpus_chunk(c0, min(N, c0 + (1 << 20)), 768, centers, dev))
probe = np.array([0, 1, N // 2, N - 1])
g0 = st.get(probe)
p_tok = torch.randint(1000, rs.vocab_size, (N, 94), device=dev, dtype=torch.int32)
p_len = torch.full((N,), 94, dtype=torch.int32, device=dev)
gq = torch.Generator(device=dev); gq.manual_seed(2)
ids = torch.randint(1000, es.vocab_size, (256, 32), generator=gq, device=dev, dtype=torch.int32)
ids[:, 0] = 101; ids[:, -1] = 102
mask = torch.ones_like(ids)
qtok = torch.randint(1000, rs.vocab_size, (256, 30), generator=gq, device=dev, dtype=torch.int32)
qlen = torch.full((256,), 30, dtype=torch.int32, device=dev)
pipe = SearchPipeline(emb, rer, st, p_tok, p_len)
q = emb.embed_dev(ids, mask, fp16=True)
s0, r0 = st.search_dev(q, 100); torch.cuda.synchronize()
print("search0 rows", r0[0, :5].tolist())
Nn.profile_enable(True)
for it in range(3):
    t0 = time.time()
    res = pipe.run(ids, mask, qtok, qlen); torch.cuda.synchronize()
    prof = Nn.profile_read(); Nn.profile_enable(True)
    print(it, f"{time.time()-t0:.3f}s scans", prof.get("cosine_scan", {}).get("launches"),
          "cand rows", res.cand_rows[0, :5].tolist(), "same as search0:", bool((res.cand_rows == r0).all().item()),
          "final", res.rows[0, :3].tolist(), "logits", res.logits[0, :3].tolist())
    print("   corpus intact:", np.array_equal(st.get(probe), g0))
q2 = emb.embed_dev(ids, mask, fp16=True)
print("embed stable:", bool((q2 == q).all().item()))
