"""CPU: the host C++ under AddressSanitizer + UndefinedBehaviorSanitizer (VERDICT r3
item 8).  `make -C super-rag_amd asan` builds every native source with the sanitizers on the host
side (-Xarch_host; the device code is untouched and never launched) and links the robustness
driver tests/native/fuzz_loaders.cpp: every truncation and a set of corruptions of a store
snapshot (.srmi) and a BM25 snapshot (.srlex), 400 random header bit flips, and invalid arguments
to the C-ABI entry points.  Each case must return an SR_ERR_* code (SR_ERR_IO for the snapshots,
before anything is allocated) with no sanitizer report.  No GPU needed."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_loaders_and_argument_validation_under_asan_ubsan(tmp_path):
    jobs = str(min(8, os.cpu_count() or 1))
    b = subprocess.run(["make", "-C", os.path.join(ROOT, "super-rag_amd"), "asan", "-j", jobs],
                       capture_output=True, text=True, timeout=1200)
    assert b.returncode == 0, b.stdout[-3000:] + b.stderr[-3000:]
    exe = os.path.join(ROOT, "super-rag_amd", "build_asan", "fuzz_loaders")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", ""))
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=600, env=env)
    out = r.stdout + r.stderr
    print(out[-2000:])
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert " 0 failures" in r.stdout
