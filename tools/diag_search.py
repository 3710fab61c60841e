"""Diagnostic: search correctness at bench scale (not part of the product)."""
import os, sys, time
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "super-rag_amd")]
import numpy as np, torch
import bench
from super_rag_amd.encoder import MODELS, Encoder, random_weights
from super_rag_amd.store import NativeStore
dev = torch.device("cuda", 0)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
es = MODELS["bge-base-en"]
emb = Encoder(es, weights=random_weights(es, 11, "hf"), max_tokens=8192)
gc = torch.Generator(device="cpu"); gc.manual_seed(0)
centers = torch.randn((1024, 768), generator=gc).to(dev)
st = NativeStore(768, capacity=N)
for c0 in range(0, N, 1 << 20):
    st.add_dev(bench.gen_corpus_chunk(c0, min(N, c0 + (1 << 20)), 768, centers, dev))
gq = torch.Generator(device=dev); gq.manual_seed(2)
ids = torch.randint(1000, es.vocab_size, (256, 32), generator=gq, device=dev, dtype=torch.int32)
ids[:, 0] = 101; ids[:, -1] = 102
mask = torch.ones_like(ids)
q = emb.embed_dev(ids, mask, fp16=False)
print("q finite", torch.isfinite(q).all().item(), "norms", q.norm(dim=1)[:4].tolist())
qn = torch.nn.functional.normalize(q, dim=1)
print("query pairwise cos min", (qn @ qn.T).min().item())
for B in (256, 32, 1):
    for k in (10, 100):
        t0 = time.time(); s, r = st.search_dev(q[:B].contiguous(), k); torch.cuda.synchronize()
        print(f"B={B} k={k} search {time.time()-t0:.3f}s rows0 {r[0,:5].tolist()} sims0 {s[0,:5].tolist()}")
nq = 8
best_s = torch.full((nq, 0), -2.0, device=dev); best_r = torch.zeros((nq, 0), dtype=torch.int64, device=dev)
for c0 in range(0, N, 1 << 20):
    x = bench.gen_corpus_chunk(c0, min(N, c0 + (1 << 20)), 768, centers, dev)
    sc = qn[:nq] @ torch.nn.functional.normalize(x, dim=1).T
    best_s = torch.cat([best_s, sc], 1)
    best_r = torch.cat([best_r, torch.arange(c0, c0 + x.shape[0], device=dev).expand(nq, -1)], 1)
    top = best_s.topk(100, dim=1); best_s, best_r = top.values, best_r.gather(1, top.indices)
print("exact rows0", best_r[0, :5].tolist(), "sims", best_s[0, :5].tolist())
print("exact sims at 10/100:", best_s[0, 9].item(), best_s[0, 99].item())
s, r = st.search_dev(q[:nq].contiguous(), 100)
for i in range(nq):
    print(i, "recall10", len(set(r[i,:10].tolist()) & set(best_r[i,:10].tolist())) / 10,
          "recall100", len(set(r[i].tolist()) & set(best_r[i].tolist())) / 100)
