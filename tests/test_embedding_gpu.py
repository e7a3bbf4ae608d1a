"""Host-sync-free embedding backward (ops/embedding.py) against the stock op."""
import pytest
import torch
import torch.nn.functional as F

from apex_example_amd.ops.embedding import Embedding

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n_idx", [1000, 16384])
def test_embedding_backward_matches_stock(dtype, n_idx):
    torch.manual_seed(0)
    emb = Embedding(30522, 256).to(dev).to(dtype)
    idx = torch.randint(0, 30522, (n_idx,), device=dev)
    idx[: n_idx // 4] = 7  # many repeats of one row
    dy = torch.randn(n_idx, 256, device=dev).to(dtype)
    emb(idx).backward(dy)
    w = emb.weight.detach().clone().requires_grad_(True)
    F.embedding(idx, w).backward(dy)
    ref = torch.zeros(30522, 256, device=dev).index_add_(0, idx, dy.float())
    scale = ref.abs().max().item()
    # ours: fp32 accumulation, one rounding to the weight dtype
    tol = 1e-5 if dtype == torch.float32 else 8e-3
    assert (emb.weight.grad.float() - ref).abs().max().item() <= tol * scale
    assert (w.grad.float() - ref).abs().max().item() <= 4 * tol * scale + 1e-6
    torch.testing.assert_close(emb(idx), F.embedding(idx, w))


def test_embedding_padding_idx_and_tied_grad():
    emb = Embedding(100, 16, padding_idx=3).to(dev)
    idx = torch.tensor([[3, 5, 3, 9]], device=dev)
    y = emb(idx)
    logits = F.linear(y, emb.weight)  # tied use, as the LM heads
    logits.sum().backward()
    w = emb.weight.detach().clone().requires_grad_(True)
    F.linear(F.embedding(idx, w, padding_idx=3), w).sum().backward()
    torch.testing.assert_close(emb.weight.grad, w.grad, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("H", [1024, 250])   # vector path / scalar path
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_embedding_backward_is_deterministic(H, dtype):
    """The default backward (csrc/hip/embedding.hip: device sort + per-run sums in
    sorted order) is bitwise reproducible and equals the fp64 sum to one rounding."""
    torch.manual_seed(1)
    V = 5000
    emb = Embedding(V, H, padding_idx=11).to(dev).to(dtype)
    idx = torch.randint(0, V, (8, 512), device=dev)
    idx[:, :64] = 42                      # a long run (512 repeats)
    idx[0, :5] = 11                       # padding ids
    dy = torch.randn(8, 512, H, device=dev).to(dtype)
    grads = []
    for _ in range(3):
        emb.weight.grad = None
        emb(idx).backward(dy)
        grads.append(emb.weight.grad.clone())
    assert all(torch.equal(grads[0], g) for g in grads[1:])
    ref = torch.zeros(V, H, dtype=torch.float64, device=dev).index_add_(
        0, idx.reshape(-1), dy.reshape(-1, H).double())
    ref[11] = 0
    err = (grads[0].double() - ref).abs().max().item() / ref.abs().max().item()
    assert err <= (1e-6 if dtype == torch.float32 else 2 ** -8), err
    assert grads[0].dtype == dtype and torch.count_nonzero(grads[0][11]) == 0


@pytest.mark.parametrize("case", ["token_type", "boundaries", "long_pad"])
def test_embedding_backward_long_runs_chunked(case):
    """Runs longer than one 256-position chunk are summed as chunk partials joined in
    order (BERT's 2-row token-type table: two runs of ~8k tokens): exact vs fp64 to one
    rounding, bitwise reproducible, including runs that start / end on chunk boundaries
    and a long padding run."""
    torch.manual_seed(2)
    H = 1024
    if case == "token_type":
        V, pad = 2, None
        idx = torch.randint(0, 2, (32, 512), device=dev)
    elif case == "boundaries":
        V, pad = 16, None
        lens = [256, 256, 257, 255, 1, 512, 768, 3, 300, 1]
        idx = torch.cat([torch.full((n,), i, dtype=torch.long) for i, n in enumerate(lens)])
        idx = idx[torch.randperm(idx.numel())].to(dev)
    else:
        V, pad = 8, 5
        idx = torch.randint(0, V, (4096,), device=dev)
        idx[:3000] = 5
    emb = Embedding(V, H, padding_idx=pad).to(dev).to(torch.bfloat16)
    dy = torch.randn(*idx.shape, H, device=dev).to(torch.bfloat16)
    grads = []
    for _ in range(2):
        emb.weight.grad = None
        emb(idx).backward(dy)
        grads.append(emb.weight.grad.clone())
    assert torch.equal(grads[0], grads[1])
    ref = torch.zeros(V, H, dtype=torch.float64, device=dev).index_add_(
        0, idx.reshape(-1), dy.reshape(-1, H).double())
    if pad is not None:
        ref[pad] = 0
        assert torch.count_nonzero(grads[0][pad]) == 0
    err = (grads[0].double() - ref).abs().max().item() / ref.abs().max().item()
    assert err <= 2 ** -8, err
