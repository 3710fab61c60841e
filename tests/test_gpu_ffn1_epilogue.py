"""GPU: the LayerNorm-folded FFN1 GEMM (`gemm_f16_lnfold_gelu` / `gemm_f8_lnfold_gelu_out8`) on
ragged row counts, every output row against a torch fp32 reference, and the rows past M untouched.

The fp16 epilogue leaves through range-checked buffer stores (one buffer resource per 16-row group,
its size ending at row M) and the fp8 one likewise (SR_GEMM_GELU_BUFST / _BUFST8): the bounds check,
not a compare, drops the rows past M of the last tile.  A guard band after row M, filled with a
sentinel, must come back unchanged.  Reference: 2 GELU(rstd (x . w - mu c) + b) with the row
statistics (mu, rstd) of the un-normalised rows and c = the folded weight's row sums (the encoder's
LN fold, oracle/encoder_ref.py restated in torch fp32).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GUARD = 48  # rows after M that must stay untouched


def _e4m3(t):
    import torch
    return t.float().clamp(-448, 448).to(torch.float8_e4m3fn)


@pytest.mark.parametrize("f8", [False, True])
@pytest.mark.parametrize("M,N", [(1317, 3072), (256 * 9 + 255, 768), (77, 1024), (256 * 64 + 77, 3072)])
def test_ffn1_ragged_rows_and_guard_band(f8, M, N):
    import torch
    from super_rag_amd import _native as NT
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(M + N + int(f8))
    K = 768
    u = torch.randn(M, K, device=dev, generator=g) * 0.7 + 0.05
    W = torch.randn(N, K, device=dev, generator=g) * 0.04
    bias = torch.randn(N, device=dev, generator=g) * 0.1
    mr = torch.stack([u.mean(1), torch.rsqrt(u.var(1, unbiased=False) + 1e-5)], 1).contiguous()
    if f8:
        X = _e4m3(u).view(torch.uint8).contiguous()
        e = torch.floor(torch.log2(448.0 / W.abs().amax(1).clamp_min(1e-30))).to(torch.int32)
        Wop = _e4m3(W * torch.exp2(e.float())[:, None]).view(torch.uint8).contiguous()
        wexp = (127 - e).to(torch.uint8).contiguous()
        Wd = Wop.view(torch.float8_e4m3fn).float() * torch.exp2(-e.float())[:, None]
        Xd = X.view(torch.float8_e4m3fn).float()
        Yall = torch.full((M + GUARD, N), 0x5A, device=dev, dtype=torch.uint8)
        wexp_p = wexp.data_ptr()
    else:
        X = u.half().contiguous()
        Wop = W.half().contiguous()
        Wd, Xd = Wop.float(), X.float()
        Yall = torch.full((M + GUARD, N), 1234.0, device=dev, dtype=torch.float16)
        wexp_p = None
    colsum = Wd.sum(1).contiguous()
    stream = torch.cuda.current_stream().cuda_stream
    NT.call_diag("sr_diag_ffn1", 0, 1 if f8 else 0, X.data_ptr(), K, Wop.data_ptr(), wexp_p,
            bias.data_ptr(), colsum.data_ptr(), mr.data_ptr(), Yall.data_ptr(), N, M, N, K, 0, stream)
    torch.cuda.synchronize()
    pre = mr[:, 1:2] * (Xd @ Wd.T - mr[:, 0:1] * colsum[None]) + bias[None]
    ref = 2.0 * torch.nn.functional.gelu(pre)
    got = Yall[:M].view(torch.float8_e4m3fn).float() if f8 else Yall[:M].float()
    rel = ((got - ref).abs() / ref.abs().clamp_min(1.0)).max().item()
    assert rel <= (0.07 if f8 else 2e-3), rel
    guard = Yall[M:].cpu().numpy()
    assert np.all(guard == (0x5A if f8 else np.float16(1234.0))), "rows past M were written"
