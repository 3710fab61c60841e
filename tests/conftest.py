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
