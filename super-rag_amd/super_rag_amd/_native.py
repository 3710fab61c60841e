"""ctypes binding of the MI355X C-ABI (include/super_rag_mi355x.h).

The library is built in-tree (``make -C super-rag_amd`` or ``__graft_entry__.build()``) into
``super_rag_amd/lib/libsrmi.so``.  There is no CPU fallback: if the library (or a GPU) is missing,
every compute entry point raises :class:`NativeUnavailableError`.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading
import time
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int32, c_int64, c_void_p

_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libsrmi.so")

SR_OK = 0
SR_ERR_INVALID = -1
SR_ERR_HIP = -2
SR_ERR_OOM = -3
SR_ERR_IO = -4
SR_ERR_STATE = -5

SR_DTYPE_F32 = 0
SR_DTYPE_F16 = 1
SR_DTYPE_FP8_E4M3 = 2
SR_POOL_CLS = 0
SR_POOL_MEAN = 1
SR_MAX_TOPK = 1024


class NativeUnavailableError(RuntimeError):
    """The HIP library is not built / not loadable, or no GPU is visible."""


class NativeError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"[{code}] {message}")
        self.code = code
        self.message = message


class EncoderConfigC(ctypes.Structure):
    _fields_ = [
        ("vocab_size", c_int), ("hidden", c_int), ("layers", c_int), ("heads", c_int),
        ("intermediate", c_int), ("max_position", c_int), ("type_vocab", c_int),
        ("ln_eps", c_float), ("position_offset", c_int), ("classifier", c_int),
        ("num_labels", c_int), ("max_tokens", c_int), ("residual_fp16", c_int),
    ]


class KernelStatC(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 64), ("launches", c_int64), ("total_ms", c_double),
                ("flops", c_double), ("bytes", c_double)]


P_I32 = POINTER(c_int32)
P_I64 = POINTER(c_int64)
P_F32 = POINTER(c_float)

# name -> (restype, argtypes); mirrors include/super_rag_mi355x.h one to one.
SIGNATURES = {
    "sr_last_error": (c_char_p, []),
    "sr_version": (c_int, []),
    "sr_device_count": (c_int, [P_I32]),
    "sr_memcpy": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_int]),
    "sr_store_create": (c_int, [c_int, c_int, c_int64, POINTER(c_void_p)]),
    "sr_store_add": (c_int, [c_void_p, c_void_p, c_int64, c_void_p]),
    "sr_store_add_dev": (c_int, [c_void_p, c_void_p, c_int, c_int64, P_I64, c_void_p]),
    "sr_store_remove": (c_int, [c_void_p, c_void_p, c_int64]),
    "sr_store_count": (c_int, [c_void_p, P_I64, P_I64]),
    "sr_store_dim": (c_int, [c_void_p, P_I32]),
    "sr_store_get": (c_int, [c_void_p, c_void_p, c_int64, c_void_p]),
    "sr_store_search": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "sr_store_search_masked": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int64, c_void_p,
                                       c_void_p]),
    "sr_store_search_sim": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int64, c_void_p,
                                    c_void_p]),
    "sr_store_search_dev": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                    c_int64, c_void_p]),
    "sr_store_set_scan_dtype": (c_int, [c_void_p, c_int]),
    "sr_store_save": (c_int, [c_void_p, c_char_p]),
    "sr_store_load": (c_int, [c_char_p, c_int, POINTER(c_void_p)]),
    "sr_store_compact": (c_int, [c_void_p, c_void_p]),
    "sr_store_destroy": (None, [c_void_p]),
    "sr_store_set_create": (c_int, [c_int, c_int, c_void_p, c_int, POINTER(c_void_p)]),
    "sr_store_set_add": (c_int, [c_void_p, c_void_p, c_int64, c_void_p]),
    "sr_store_set_remove": (c_int, [c_void_p, c_void_p, c_int64]),
    "sr_store_set_count": (c_int, [c_void_p, P_I64, P_I64, P_I32]),
    "sr_store_set_get": (c_int, [c_void_p, c_void_p, c_int64, c_void_p]),
    "sr_store_set_search": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int64, c_void_p,
                                    c_void_p]),
    "sr_store_set_set_scan_dtype": (c_int, [c_void_p, c_int]),
    "sr_store_set_destroy": (None, [c_void_p]),
    "sr_lex_create": (c_int, [c_int, c_float, c_float, POINTER(c_void_p)]),
    "sr_lex_add": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, P_I64]),
    "sr_lex_remove": (c_int, [c_void_p, c_void_p, c_int64]),
    "sr_lex_stats": (c_int, [c_void_p, P_I64, P_I64, P_I64, P_I64, POINTER(c_double)]),
    "sr_lex_search": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int64,
                              c_void_p, c_void_p]),
    "sr_lex_totals": (c_int, [c_void_p, P_I64, P_I64]),
    "sr_lex_df": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "sr_lex_search_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                  c_void_p, c_int64, c_void_p]),
    "sr_lex_search_global": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int64,
                                     c_void_p, c_void_p, c_void_p]),
    "sr_lex_query_stats_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p,
                                       c_void_p]),
    "sr_lex_search_tok_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                      c_void_p, c_void_p, c_int64, c_void_p]),
    "sr_lex_save": (c_int, [c_void_p, c_char_p]),
    "sr_lex_load": (c_int, [c_char_p, c_int, POINTER(c_void_p)]),
    "sr_lex_compact": (c_int, [c_void_p, c_void_p]),
    "sr_lex_destroy": (None, [c_void_p]),
    "sr_rrf_fuse": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_double, c_int,
                            c_void_p, c_void_p, c_int]),
    "sr_rrf_fuse_dev": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_double, c_int,
                                c_void_p, c_void_p, c_int, c_void_p]),
    "sr_hybrid_search": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                 c_int, c_int, c_double, c_void_p, c_int64, c_void_p, c_void_p]),
    "sr_topk_merge_dev": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                                  c_void_p, c_int, c_void_p]),
    "sr_encoder_create": (c_int, [POINTER(EncoderConfigC), c_int, POINTER(c_void_p)]),
    "sr_encoder_set_weight": (c_int, [c_void_p, c_char_p, c_void_p, c_int64]),
    "sr_encoder_ready": (c_int, [c_void_p]),
    "sr_encoder_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                   c_void_p]),
    "sr_encoder_forward_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                       c_int, c_void_p, c_int, c_int, c_void_p]),
    "sr_cross_score": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "sr_cross_score_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                   c_void_p, c_void_p]),
    "sr_encoder_set_fp8": (c_int, [c_void_p, c_int]),
    "sr_encoder_destroy": (None, [c_void_p]),
    "sr_build_pairs_dev": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                   c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                   c_void_p, c_void_p, c_int, c_void_p]),
    "sr_rerank_select_dev": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "sr_profile_enable": (c_int, [c_int]),
    "sr_profile_read": (c_int, [POINTER(KernelStatC), c_int, P_I32]),
    "sr_lex_search_global_fixed": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p,
                                           c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
}

# The diagnostic surface (include/super_rag_mi355x_diag.h), exported by libsrmi_diag.so only:
# single-kernel parity entry points, timing-only variants and the HBM copy yardstick.
DIAG_SIGNATURES = {
    "sr_diag_gemm": (c_int, [c_int, c_int, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64,
                             c_void_p, c_int64, c_int, c_int, c_int, c_int, c_void_p]),
    "sr_diag_ffn1": (c_int, [c_int, c_int, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_void_p, c_void_p, c_int64, c_int, c_int, c_int, c_int, c_void_p]),
    "sr_diag_attention": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                  c_int, c_int, c_void_p]),
    "sr_diag_copy": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p]),
    "sr_diag_ffn1_stamps": (c_int, [c_int, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_int64, c_int, c_int, c_int, c_void_p, c_int,
                                    c_void_p]),
    "sr_diag_gemm_stats": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64,
                                   c_void_p, c_int64, c_int, c_int, c_int, c_void_p, c_int,
                                   c_void_p]),
    "sr_diag_qkv_attention_stamps": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
                                             c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                                             c_int, c_void_p]),
    "sr_diag_gemm_lnr_stats": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64,
                                       c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_int,
                                       c_void_p, c_int, c_void_p]),
    "sr_diag_gemm_lnr_stats_stamps": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64,
                                              c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_int,
                                              c_void_p, c_void_p, c_int, c_void_p]),
    "sr_diag_mfma_rate": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "sr_diag_gemm_stats_y8": (c_int, [c_int, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64,
                                      c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int, c_int,
                                      c_int, c_void_p, c_int, c_void_p]),
}

_lib = None
_diag = None

_gates: dict = {}
_gates_lock = threading.Lock()


class _DeviceGate:
    """The per-device lock of device_gate and the time it was held, per stage."""

    def __init__(self):
        self.lock = threading.Lock()
        self.busy: dict = {}    # stage -> [seconds held, holds]

    @contextlib.contextmanager
    def hold(self, stage: str):
        with self.lock:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                b = self.busy.setdefault(stage, [0.0, 0])
                b[0] += time.perf_counter() - t0
                b[1] += 1


def device_gate(device: int, stage: str = "device"):
    """Context manager: one lock per device, held by the coalesced request paths (embed_query,
    connector search, rerank scoring) around their device calls.  Without it, a concurrent small
    batch (a 12-layer embed of a few queries: ~100 short kernels) interleaves kernel by kernel with
    a large rerank batch on the same GPU, so each of its kernels waits for a ~1 ms rerank kernel;
    with it, each stage's batch runs back to back and the waiting requests join the next, larger
    batch.  The time held is kept per stage (gate_busy: the device's busy time by stage, since the
    calls synchronise before they return)."""
    g = _gates.get(device)
    if g is None:
        with _gates_lock:
            g = _gates.setdefault(device, _DeviceGate())
    return g.hold(stage)


@contextlib.contextmanager
def devices_gate(devices, stage: str = "device"):
    """device_gate over several devices (a collection sharded over them): every device's gate,
    taken in ascending device order (one global order, so two multi-device holders cannot
    deadlock), each charged the hold time of `stage`."""
    with contextlib.ExitStack() as st:
        for d in sorted(set(int(x) for x in devices)):
            st.enter_context(device_gate(d, stage))
        yield


def gate_busy() -> dict:
    """{device: {stage: (seconds held, holds)}} accumulated by device_gate."""
    return {d: {k: (v[0], v[1]) for k, v in g.busy.items()} for d, g in list(_gates.items())}


_lock = threading.Lock()


def library_path() -> str:
    return os.environ.get("SUPER_RAG_AMD_LIB", _LIB_PATH)


def load() -> ctypes.CDLL:
    """Load (once) and return the native library; raise NativeUnavailableError if absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64.so.7.  If this
        # library is loaded first, the dynamic loader binds /opt/rocm's copy and a later
        # torch.cuda init fails with "No HIP GPUs are available" (measured on the MI355X box);
        # importing torch first makes both bind the same, already-loaded runtime.
        try:
            import torch  # noqa: F401
        except Exception:  # noqa: BLE001 - torch is optional for the host-buffer entry points
            pass
        path = library_path()
        if not os.path.exists(path):
            raise NativeUnavailableError(
                f"MI355X native library not built: {path} (run __graft_entry__.build() or "
                f"`make -C super-rag_amd`)")
        try:
            lib = ctypes.CDLL(path)  # CDLL releases the GIL around every call
        except OSError as e:
            raise NativeUnavailableError(f"cannot load {path}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def diag_library_path() -> str:
    return os.environ.get("SUPER_RAG_AMD_DIAG_LIB",
                          os.path.join(os.path.dirname(library_path()), "libsrmi_diag.so"))


def load_diag() -> ctypes.CDLL:
    """The diagnostic library libsrmi_diag.so (the product sources + sr_diag_*; tests of single
    kernels, tools/, bench.py's measured peaks).  Never needed by the product path."""
    global _diag
    if _diag is not None:
        return _diag
    with _lock:
        if _diag is not None:
            return _diag
        try:
            import torch  # noqa: F401  (one HIP runtime per process, as in load())
        except Exception:  # noqa: BLE001
            pass
        path = diag_library_path()
        if not os.path.exists(path):
            raise NativeUnavailableError(f"diagnostic library not built: {path} (`make -C super-rag_amd`)")
        try:
            lib = ctypes.CDLL(path)
        except OSError as e:
            raise NativeUnavailableError(f"cannot load {path}: {e}") from e
        for name, (res, args) in {**SIGNATURES, **DIAG_SIGNATURES}.items():
            # (an A/B variant built from older sources may lack a newer diagnostic: skip it)
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        _diag = lib
        return lib


def call_diag(name: str, *args) -> None:
    """Call an sr_diag_* entry point of libsrmi_diag.so (errors from its own sr_last_error)."""
    lib = load_diag()
    code = getattr(lib, name)(*args)
    if code != SR_OK:
        msg = lib.sr_last_error()
        raise NativeError(code, msg.decode("utf-8", "replace") if msg else "unknown error")


def check(code: int) -> None:
    if code != SR_OK:
        msg = load().sr_last_error()
        raise NativeError(code, msg.decode("utf-8", "replace") if msg else "unknown error")


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args))


def device_count() -> int:
    n = c_int32(0)
    call("sr_device_count", ctypes.byref(n))
    return int(n.value)


def require_gpu() -> None:
    if device_count() < 1:
        raise NativeUnavailableError("no HIP device visible: the MI355X hot path needs a GPU")


def ptr(a) -> int:
    """Data pointer of a numpy array (host) or torch tensor (host or device)."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    return a.ctypes.data


def stream_handle(stream=None) -> int | None:
    """hipStream_t of a torch stream (default: the current stream of the current device)."""
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


def profile_enable(on: bool) -> None:
    call("sr_profile_enable", 1 if on else 0)


def profile_read() -> dict:
    buf = (KernelStatC * 256)()
    n = c_int32(0)
    call("sr_profile_read", buf, 256, ctypes.byref(n))
    out = {}
    for i in range(n.value):
        s = buf[i]
        out[s.name.decode()] = {"launches": int(s.launches), "total_ms": float(s.total_ms),
                                "flops": float(s.flops), "bytes": float(s.bytes)}
    return out
