"""Every tensor-taking ``torch.ops.dph`` operator has a fake (meta) implementation, so FakeTensor tracing,
torch.export and meta-device construction work through the framework's kernels (ops/_meta.py).  CPU only: the
extension loads without a GPU and fake kernels never launch anything."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

# resource-management / configuration ops with no tensor arguments (catch-all kernels, nothing to trace)
NO_TENSOR_OPS = {"gemm_tn_tail_", "gemm_tn_plan_info", "car_create", "car_ipc_handle", "car_open",
                 "car_status", "car_destroy", "car_agreed", "attn_variant", "gemm_nt_variant", "gemm1_lds",
                 "c3w_round"}


@pytest.fixture(scope="module")
def dph_ops():
    from distributed_pytorch_hpc_amd.ops import _lib

    if not _lib.load():
        pytest.skip(f"native extension not loadable: {_lib._error}")
    import distributed_pytorch_hpc_amd.ops._meta  # noqa: F401
    return sorted({n.split("::")[1].split(".")[0] for n in torch._C._dispatch_get_all_op_names()
                   if n.startswith("dph::")})


def test_every_tensor_op_has_a_fake(dph_ops):
    from torch._library.simple_registry import singleton

    assert len(dph_ops) > 30
    missing = []
    for name in dph_ops:
        if name in NO_TENSOR_OPS:
            continue
        entry = singleton.find(f"dph::{name}")
        if entry.fake_impl.kernel is None:
            missing.append(name)
    assert not missing, f"ops without a fake implementation: {missing}"


def test_fakes_produce_kernel_shapes(dph_ops):
    d = torch.ops.dph
    with FakeTensorMode():
        q = torch.empty(2, 128, 4, 64, dtype=torch.bfloat16)
        o, lse = d.flash_attn_fwd(q, q, q, 0.125, True)
        assert o.shape == q.shape and lse.shape == (2, 4, 128) and lse.dtype == torch.float32
        dq, dk, dv = d.flash_attn_bwd(o, q, q, q, o, lse, 0.125, True)
        assert dq.shape == dk.shape == dv.shape == q.shape
        ids = torch.empty(2, 16, dtype=torch.long)
        tab = torch.empty(512, 64, dtype=torch.bfloat16)
        assert d.embedding_fwd(ids, tab, 0).shape == (2, 16, 64)
        assert d.embedding_bwd(ids, torch.empty(2, 16, 64, dtype=torch.bfloat16), 512, 0).shape == (512, 64)
        logits = torch.empty(32, 512, dtype=torch.bfloat16)
        loss, lse2 = d.cross_entropy_fwd(logits, torch.empty(32, dtype=torch.long), torch.empty(1), -100, True, 0.0)
        assert loss.shape == lse2.shape == (32,)
        y, yt, s = d.fp8_quantize(torch.empty(128, 64, dtype=torch.bfloat16), 0, True, True)
        assert y.shape == (128, 64) and yt.shape == (64, 128) and y.dtype == torch.float8_e4m3fn and s.dim() == 0
        assert d.skinny_linear(torch.empty(4, 256, dtype=torch.bfloat16),
                               torch.empty(512, 256, dtype=torch.bfloat16)).shape == (4, 512)
        assert d.swiglu_fwd(torch.empty(8, 64, dtype=torch.bfloat16)).shape == (8, 32)
