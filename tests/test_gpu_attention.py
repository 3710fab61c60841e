"""GPU parity of the K5 attention kernels (through the diagnostic library's sr_diag_attention, libsrmi_diag.so) against
a torch fp32 reference: ctx = softmax(Q K^T / sqrt(d_h) + key-padding mask) V per head, for the
first Sq query rows of each sequence.

Covers both kernels (64-key tiles; whole head in LDS with transposed V reads, and its SPLIT
staging at S_pad = 128, the 8-wave form and its key-block STREAM staging at S_pad = 512; variant
-1 = the automatic choice), ragged masks,
S not a multiple of 16 / 32, S > 128 (online softmax across 128-key blocks), Sq = 1 (the CLS-only
last layer), fully masked rows except the first key.  Tolerance: |ctx - ref| <= 4e-3 (fp16 P and
output, fp32 statistics; |ref| <= max|V| ~ 1).
"""
import pytest

pytestmark = pytest.mark.gpu


def _run(variant, B, S, Sq, heads, dh=64, seed=0, lens=None):
    import torch
    from super_rag_amd import _native as NT
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(seed)
    d = heads * dh
    qkv = (torch.randn(B * S, 3 * d, device=dev, generator=g) * 1.5).half()
    if lens is None:
        lens = torch.randint(1, S + 1, (B,), device=dev, generator=g)
    mask = (torch.arange(S, device=dev)[None] < lens[:, None]).int().contiguous()
    ctx = torch.full((B * Sq, d), float("nan"), device=dev, dtype=torch.float16)
    NT.call_diag("sr_diag_attention", variant, qkv.data_ptr(), mask.data_ptr(), ctx.data_ptr(), B, S, Sq,
            d, heads, 0, torch.cuda.current_stream().cuda_stream)
    x = qkv.float().view(B, S, 3, heads, dh)
    q, k, v = x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)
    sc = q @ k.transpose(-1, -2) / dh ** 0.5
    sc = sc.masked_fill(mask[:, None, None, :] == 0, float("-inf"))
    ref = (torch.softmax(sc, -1) @ v).transpose(1, 2)[:, :Sq].reshape(B * Sq, d)
    torch.cuda.synchronize()
    return (ctx.float() - ref).abs().max().item()


@pytest.mark.parametrize("variant", [0, 1, 2, 3, -1])
@pytest.mark.parametrize("S,Sq", [(128, 128), (128, 1), (32, 32), (100, 100), (7, 7), (200, 200),
                                  (512, 512), (300, 1), (130, 130),
                                  # K5b SPLIT boundaries (S_pad == 128 and Sq > 96): first / last
                                  # S of the split range, the last query tile partly stored, and
                                  # Sq = 96 (non-split: wave 3 idle)
                                  (97, 97), (128, 97), (128, 96), (120, 110),
                                  # K5d (auto) / K5b STREAM (variant 3): 8 waves, S_pad = 512, Sq > 480
                                  (500, 500), (512, 481), (512, 480)])
def test_attention_vs_torch(variant, S, Sq):
    err = _run(variant, 6, S, Sq, heads=3, seed=S * 7 + Sq)
    assert err <= 4e-3, f"variant {variant} S={S} Sq={Sq}: max|err| {err:.3e}"


def test_attention_single_key_rows():
    import torch
    lens = torch.tensor([1, 1, 2, 128], device="cuda")
    for variant in (0, 1, 2, 3, -1):
        err = _run(variant, 4, 128, 128, heads=2, seed=3, lens=lens)
        assert err <= 4e-3, f"variant {variant}: max|err| {err:.3e}"


@pytest.mark.parametrize("S,Sq", [(512, 512), (500, 500), (512, 481)])
def test_attention_k5d_persistent_walkers(S, Sq):
    # K5d (auto at S_pad = 512, every query): 600 (sequence, head) tiles over 256 walkers, so
    # walkers take 2-3 tiles and every key block, query panel and key bias is refilled from the
    # next tile during pass B; ragged lengths per sequence.  Must equal K5b STREAM (variant 3) bit
    # for bit (same block code and operation order) and the torch reference within 4e-3.
    import torch
    from super_rag_amd import _native as NT
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(S + Sq)
    B, heads, dh = 150, 4, 64
    d = heads * dh
    qkv = (torch.randn(B * S, 3 * d, device=dev, generator=g) * 1.5).half()
    lens = torch.randint(1, S + 1, (B,), device=dev, generator=g)
    lens[::7] = S
    mask = (torch.arange(S, device=dev)[None] < lens[:, None]).int().contiguous()
    outs = {}
    for variant in (3, -1):
        ctx = torch.full((B * Sq, d), float("nan"), device=dev, dtype=torch.float16)
        NT.call_diag("sr_diag_attention", variant, qkv.data_ptr(), mask.data_ptr(), ctx.data_ptr(), B, S,
                Sq, d, heads, 0, torch.cuda.current_stream().cuda_stream)
        outs[variant] = ctx
    torch.cuda.synchronize()
    assert torch.equal(outs[-1], outs[3])
    x = qkv.float().view(B, S, 3, heads, dh)
    q, k, v = x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)
    sc = q @ k.transpose(-1, -2) / dh ** 0.5
    sc = sc.masked_fill(mask[:, None, None, :] == 0, float("-inf"))
    ref = (torch.softmax(sc, -1) @ v).transpose(1, 2)[:, :Sq].reshape(B * Sq, d)
    assert (outs[-1].float() - ref).abs().max().item() <= 4e-3
