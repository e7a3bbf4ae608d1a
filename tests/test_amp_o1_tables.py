"""O1 cast-table parity (upstream test_basic_casts.py,
test_promotion.py): every entry of Apex's FP16 / FP32 / CASTS / SEQUENCE_CASTS /
BANNED tables (amp/lists/) is called under O1 and its output dtype checked
against Apex's policy, for fp16 and bf16.

On this CPU host the CUDA autocast policy is exercised with FakeTensorMode
"cuda" tensors (the autocast dispatch key runs; no device is touched); the GPU
test repeats the audit on real MI355X tensors through amp.initialize.
"""
import pytest
import torch
import torch.nn.functional as F

from apex_example_amd.amp import amp as amp_mod
from apex_example_amd.amp.lists import audit as A


@pytest.fixture
def o1():
    handles = []

    def start(dtype, allow_banned=False):
        h = amp_mod.init(dtype=dtype, device_type="cuda", allow_banned=allow_banned)
        handles.append(h)
        return h
    yield start
    amp_mod.deinit()
    torch.set_autocast_enabled("cuda", False)
    from apex_example_amd.amp._amp_state import _amp_state
    _amp_state.handle = None


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_every_apex_table_entry_matches_under_o1_fake_cuda(o1, dtype):
    o1(dtype)
    bad = A.audit("cuda", dtype, fake=True)
    assert bad == [], bad


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_override_list_is_exactly_the_autocast_difference(dtype):
    """Plain autocast (no overrides) disagrees with Apex on precisely the entries
    amp.amp.APEX_POLICY_OVERRIDES patches - no more, no fewer."""
    torch.set_autocast_dtype("cuda", dtype)
    torch.set_autocast_enabled("cuda", True)
    try:
        bad = A.audit("cuda", dtype, fake=True)
    finally:
        torch.set_autocast_enabled("cuda", False)
    want = [e for e in amp_mod.APEX_POLICY_OVERRIDES if e not in A.FAKE_UNVERIFIABLE]
    assert sorted((ns, n) for ns, n, *_ in bad) == sorted(want)


def test_every_table_entry_has_a_recipe():
    rec = A._recipes("cpu")
    missing = [(ns, n) for ns, n, _ in A._tables() if (ns, n) not in rec]
    assert missing == []
    # the audit covers all four Apex tables of all three namespaces
    kinds = {k for _, _, k in A._tables()}
    assert kinds == {"fp16", "fp32", "promote", "sequence", "banned"}
    assert len(A._tables()) > 150


def test_overrides_only_active_under_autocast_and_restored(o1):
    x = torch.randn(8, dtype=torch.bfloat16)
    orig_std = torch.std
    o1(torch.float16)
    assert torch.std is not orig_std
    # autocast off in this region: the wrapper is a pass-through
    with torch.autocast("cuda", enabled=False):
        assert torch.std(x).dtype == torch.bfloat16
    amp_mod.deinit()
    assert torch.std is orig_std and F.gelu.__module__ != "functools"


def test_banned_function_raises_and_allow_banned(o1):
    from torch._subclasses.fake_tensor import FakeTensorMode

    o1(torch.float16)
    with FakeTensorMode():
        p = torch.rand(4, 4, device="cuda").to(torch.float16)
        with pytest.raises(RuntimeError):
            F.binary_cross_entropy(p, p)
    amp_mod.deinit()
    o1(torch.float16, allow_banned=True)
    with FakeTensorMode():
        p = torch.rand(4, 4, device="cuda").to(torch.float16)
        assert F.binary_cross_entropy(p, p).dtype == torch.float32


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_every_apex_table_entry_matches_under_o1_gpu(dtype):
    from apex_example_amd import amp

    model = torch.nn.Linear(4, 4).cuda()
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    amp.initialize(model, opt, opt_level="O1", half_dtype=dtype, verbosity=0)
    try:
        bad = A.audit("cuda", dtype, fake=False)
    finally:
        amp_mod.deinit()
    assert bad == [], bad
