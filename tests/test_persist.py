"""CPU: checkpoint / resume of connector collections (super_rag_amd/persist.py).

The reference's ingest adds one document's chunks per call (llm/embed/embedding_utils.py:95) and
deletes by context_ids (index/vector_and_full_text_index.py:110-129); SeekDB persisted them
server-side.  Here every mutation is journaled: bytes written per add are proportional to the rows
added (not to the collection), a restart replays base + journal to the identical state, and the
snapshot files are written tmp + rename with a generation that restore checks.
"""
import json
import os

import numpy as np
import pytest

from doubles import NumpyLex, NumpyStore, hash_vec


@pytest.fixture
def doubles():
    from super_rag_amd import vectorstore
    vectorstore.set_store_backend(lambda dim, dev: NumpyStore(dim, dev), NumpyStore.load)
    vectorstore.set_lex_backend(lambda dev: NumpyLex(dev), NumpyLex.load)
    vectorstore._collections.clear()
    yield vectorstore
    vectorstore._collections.clear()
    vectorstore.set_store_backend(vectorstore._native_store, vectorstore._native_load)
    vectorstore.set_lex_backend(vectorstore._native_lex, vectorstore._native_lex_load)


def _node(i, dim=8):
    from super_rag_amd.models import TextNode
    return TextNode(text=f"doc {i} chunk", metadata={"i": i, "source": f"f{i}.md"},
                    embedding=hash_vec(f"doc {i}", dim))


def _state(con, queries):
    from super_rag_amd.models import QueryWithEmbedding
    out = []
    for q in queries:
        r = con.search(QueryWithEmbedding(query=q, top_k=7, embedding=hash_vec(q)))
        out.append([(d.text, round(d.score, 12), json.dumps(d.metadata, sort_keys=True)) for d in r.results])
    return out


def _written(path):
    return sum(os.path.getsize(os.path.join(path, f)) for f in os.listdir(path))


def test_single_node_adds_write_bytes_proportional_to_rows(doubles, tmp_path):
    ctx = {"collection": "jr", "snapshot_dir": str(tmp_path), "checkpoint_ratio": 1e9}
    con = doubles.MI355XVectorStoreConnector(ctx)
    con.add([_node(0)])                              # first add commits generation 1
    base = _written(tmp_path)
    sizes = []
    ids = []
    for i in range(1, 1001):                         # 1,000 single-node adds (one chunk each)
        before = _written(tmp_path)
        ids += con.add([_node(i)])
        sizes.append(_written(tmp_path) - before)
    # every add appends its own row only: 8 fp32 (32 B) + one JSON line, never the corpus
    assert max(sizes) < 400 and min(sizes) > 32
    assert abs(np.mean(sizes[-100:]) - np.mean(sizes[:100])) < 8   # flat in the collection size
    assert _written(tmp_path) < base + 400 * 1000
    meta = json.load(open(tmp_path / "jr.json"))
    assert meta["gen"] == 1 and meta["n_rows"] == 1             # the base was not rewritten
    # a few deletes are journaled too
    con.delete(ids=ids[10:13])
    queries = ["doc 12", "doc 500", "doc 999", "doc 3"]
    want = _state(con, queries)
    doubles._collections.clear()                                # restart
    con2 = doubles.MI355XVectorStoreConnector(ctx)
    assert _state(con2, queries) == want
    c = doubles._get("jr")
    assert len(c.ids) == 1001 and c.ids[11] is None and c.store.count() == (1001, 998)


def test_compaction_and_journal_growth_write_a_new_base(doubles, tmp_path):
    ctx = {"collection": "cb", "snapshot_dir": str(tmp_path), "checkpoint_ratio": 0.0}
    con = doubles.MI355XVectorStoreConnector(ctx)
    ids = con.add([_node(i) for i in range(20)])
    for i in range(20, 24):
        ids += con.add([_node(i)])
    assert json.load(open(tmp_path / "cb.json"))["gen"] == 1   # journal well below 64 MiB
    con.delete(ids=ids[:15])                                    # > 50 % dead: compaction
    meta = json.load(open(tmp_path / "cb.json"))
    assert meta["gen"] == 2 and meta["n_rows"] == 9
    assert sorted(os.listdir(tmp_path)) == ["cb.g2.srmi", "cb.json"]   # journal reset, gen 1 gone
    want = _state(con, ["doc 20", "doc 3"])
    doubles._collections.clear()
    assert _state(doubles.MI355XVectorStoreConnector(ctx), ["doc 20", "doc 3"]) == want


def test_torn_journal_tail_and_stale_generations_are_ignored(doubles, tmp_path):
    ctx = {"collection": "tt", "snapshot_dir": str(tmp_path)}
    con = doubles.MI355XVectorStoreConnector(ctx)
    con.add([_node(i) for i in range(5)])
    con.add([_node(5)])
    want = _state(con, ["doc 5", "doc 1"])
    with open(tmp_path / "tt.log", "a") as f:                   # crash mid-append
        f.write('{"g": 1, "op": "add", "row": 6, "n": 1, "off": 0, "ids": ["x"')
    with open(tmp_path / "tt.log", "r") as f:
        lines = f.readlines()
    with open(tmp_path / "tt.log", "w") as f:                   # a leftover of generation 0
        f.write(json.dumps({"g": 0, "op": "del", "rows": [0, 1, 2]}) + "\n")
        f.writelines(lines)
    doubles._collections.clear()
    con2 = doubles.MI355XVectorStoreConnector(ctx)
    assert _state(con2, ["doc 5", "doc 1"]) == want
    assert doubles._get("tt").store.count() == (6, 6)
    # the recovered collection keeps journaling: the torn fragment must not swallow the next add
    new_ids = con2.add([_node(6)])
    con2.delete(ids=[new_ids[0]])
    con2.add([_node(7)])
    want2 = _state(con2, ["doc 7", "doc 5", "doc 1"])
    doubles._collections.clear()
    con3 = doubles.MI355XVectorStoreConnector(ctx)
    assert _state(con3, ["doc 7", "doc 5", "doc 1"]) == want2
    assert doubles._get("tt").store.count() == (8, 7)
    with open(tmp_path / "tt.log", "rb") as f:
        assert all(json.loads(l) for l in f.read().splitlines())   # every line parses again


def test_base_bytes_counts_shard_files(tmp_path):
    """A sharded collection's <name>.g<gen>.srmi is a small manifest: the checkpoint ratio must see
    the shard stores and row tables too."""
    from super_rag_amd.persist import Journal
    j = Journal(str(tmp_path), "sh")
    j.gen = 3
    (tmp_path / "sh.g3.srmi").write_bytes(b"m" * 10)
    (tmp_path / "sh.g3.srmi.s0").write_bytes(b"x" * 1000)
    (tmp_path / "sh.g3.srmi.s1").write_bytes(b"x" * 2000)
    (tmp_path / "sh.g3.srmi.rows.npz").write_bytes(b"r" * 300)
    (tmp_path / "sh.g3.srlex").write_bytes(b"l" * 40)
    (tmp_path / "sh.g2.srmi.s0").write_bytes(b"o" * 99999)         # another generation
    (tmp_path / "other.g3.srmi").write_bytes(b"o" * 99999)         # another collection
    assert j.base_bytes() == 10 + 1000 + 2000 + 300 + 40


def test_restore_refuses_an_inconsistent_snapshot(doubles, tmp_path):
    ctx = {"collection": "bad", "snapshot_dir": str(tmp_path)}
    con = doubles.MI355XVectorStoreConnector(ctx)
    con.add([_node(i) for i in range(4)])
    meta = json.load(open(tmp_path / "bad.json"))
    meta["ids"].append("extra")
    meta["n_rows"] = 5
    json.dump(meta, open(tmp_path / "bad.json", "w"))
    doubles._collections.clear()
    with pytest.raises(IOError, match="inconsistent"):
        doubles.MI355XVectorStoreConnector(ctx)


def test_round1_layout_is_migrated(doubles, tmp_path):
    """<name>.srmi + <name>.json without a generation (the round-1 snapshot) still restores and
    is rewritten as generation 1 of the journaled layout."""
    s = NumpyStore(8)
    s.add(np.asarray([hash_vec(f"doc {i}") for i in range(3)], np.float32))
    s.save(str(tmp_path / "old.srmi"))
    json.dump({"dim": 8, "ids": ["a", "b", "c"], "texts": ["t0", "t1", "t2"],
               "metadatas": [None, {"k": 1}, None]}, open(tmp_path / "old.json", "w"))
    con = doubles.MI355XVectorStoreConnector({"collection": "old", "snapshot_dir": str(tmp_path)})
    assert sorted(os.listdir(tmp_path)) == ["old.g1.srmi", "old.json"]
    con.delete(ids=["b"])
    doubles._collections.clear()
    doubles.MI355XVectorStoreConnector({"collection": "old", "snapshot_dir": str(tmp_path)})
    assert doubles._get("old").ids == ["a", None, "c"]


def test_fulltext_collection_replays_the_lexical_index(doubles, tmp_path):
    from super_rag_amd.models import TextNode
    ctx = {"collection": "lx", "snapshot_dir": str(tmp_path), "fulltext": True}
    con = doubles.MI355XVectorStoreConnector(ctx)
    words = ["apple pie", "banana split", "cherry tart", "apple crumble", "grape juice"]
    ids = [con.add([TextNode(text=w, metadata={}, embedding=hash_vec(w))])[0] for w in words]
    con.delete(ids=[ids[0]])
    want = [d.text for d in con.fulltext_search("apple", 5)]
    assert want == ["apple crumble"]
    doubles._collections.clear()
    con2 = doubles.MI355XVectorStoreConnector(ctx)
    assert [d.text for d in con2.fulltext_search("apple", 5)] == want
    assert [d.text for d in con2.fulltext_search("banana grape", 5)] == \
        [d.text for d in con.fulltext_search("banana grape", 5)]
    con2.delete_collection()
    assert os.listdir(tmp_path) == []
