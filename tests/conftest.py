import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "super-rag_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")

# Seeded random weights and the hashing tokenizer are an explicit opt-in of tests and benchmarks
# (encoder.synthetic_allowed); tests of the product-path refusal delete the variable.
os.environ.setdefault("SUPER_RAG_AMD_SYNTHETIC", "1")


# Parity-critical files first (under `pytest -x` a late failure in a long perf-study
# test must not hide them): the reference's own cosine fixtures, every BASELINE config, the
# reference flow and the drop-in boundary run before the kernel-level studies.
_FIRST = ("test_gpu_cosine_fixtures.py", "test_gpu_configs.py", "test_gpu_rerank_fidelity.py",
          "test_gpu_flow.py", "test_gpu_boundary.py")


def pytest_collection_modifyitems(session, config, items):
    def rank(item):
        name = os.path.basename(str(item.fspath))
        return _FIRST.index(name) if name in _FIRST else len(_FIRST)
    items.sort(key=rank)   # stable: file order and in-file order kept otherwise
