"""Split-bf16 full-softmax head (precision f32x9 / f32x6, csrc/head_split.hip)
against an fp64 torch reference of the reference's nn.Linear + CrossEntropy
(GRU4Rec/model.py:58-60,80,121): the same contract and tolerances as the
native fp32 path in test_gpu_kernels.py::test_head_forward_backward."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TERMS = {"f32x9": 9, "f32x6": 6}


def C():
    import recommenders.hip as h
    return h


def st():
    return C().stream_ptr()


@pytest.mark.parametrize("precision", ["f32x9", "f32x6"])
@pytest.mark.parametrize("B,A,HF", [(64, 1000, 32), (128, 3001, 64), (96, 4133, 128), (64, 777, 256)])
def test_split_head_forward_matches_fp64(precision, B, A, HF):
    torch.manual_seed(B + A + HF)
    dev = "cuda"
    h = torch.randn(B, HF) * 0.5
    W = torch.randn(A, HF) * (HF ** -0.5)
    b = torch.randn(A) * 0.1
    tgt = torch.randint(0, A, (B,))
    hd, Wd, bd, td = h.to(dev), W.to(dev), b.to(dev), tgt.to(dev)
    ldz = (B + 3) // 4 * 4
    pb = C().load_library().rg_partial_block()
    nJ = (A + pb - 1) // pb
    ZT = torch.full((A, ldz), float("nan"), device=dev)
    pm = torch.zeros(nJ, B, device=dev)
    ps = torch.zeros(nJ, B, device=dev)
    pa = torch.zeros(nJ, B, dtype=torch.int32, device=dev)
    work = torch.empty(C().call("rg_head_work_bytes", B, HF), dtype=torch.uint8, device=dev)
    C().call("rg_head_fwd_x", hd.data_ptr(), Wd.data_ptr(), bd.data_ptr(), B, A, HF, TERMS[precision],
             ZT.data_ptr(), ldz, pm.data_ptr(), ps.data_ptr(), pa.data_ptr(), 1, work.data_ptr(), st())
    Zref = h.double() @ W.double().t() + b.double()
    torch.testing.assert_close(ZT[:, :B].t().cpu().double(), Zref, rtol=0, atol=1e-5)
    work2 = torch.zeros(3 * min(128, nJ) * B, device=dev)
    lse = torch.zeros(B, device=dev)
    amax = torch.zeros(B, dtype=torch.int32, device=dev)
    lrow = torch.zeros(B, device=dev)
    mx = torch.zeros(B, device=dev)
    C().call("rg_lse_combine", pm.data_ptr(), ps.data_ptr(), pa.data_ptr(), B, nJ, work2.data_ptr(), ZT.data_ptr(),
             ldz, td.data_ptr(), A, lse.data_ptr(), amax.data_ptr(), lrow.data_ptr(), mx.data_ptr(), st())
    torch.testing.assert_close(lse.cpu().double(), torch.logsumexp(Zref, 1), rtol=0, atol=2e-5)
    Zg = ZT[:, :B].t().cpu()
    np.testing.assert_array_equal(mx.cpu().numpy(), Zg.max(1).values.numpy())
    assert torch.equal(amax.cpu().long(), torch.argmax(Zg, 1))  # first maximum of the stored logits
    ce = torch.nn.functional.cross_entropy(Zref, tgt, reduction="none")
    torch.testing.assert_close(lrow.cpu().double(), ce, rtol=0, atol=2e-5)


def test_split_head_forward_no_store_and_ties():
    """Zᵀ not stored (argmax path) and planted exact ties: the partials give
    the first (lowest-index) maximum, like torch.argmax."""
    dev = "cuda"
    B, A, HF = 64, 2000, 128
    torch.manual_seed(3)
    h = torch.randn(B, HF) * 0.5
    W = torch.randn(A, HF) * 0.05
    W[1500] = W[7]   # duplicated rows -> exactly tied logits
    W[1999] = W[300]
    b = torch.zeros(A)
    b[7] = b[1500] = b[300] = b[1999] = 5.0  # make the tied items the maxima
    pb = C().load_library().rg_partial_block()
    nJ = (A + pb - 1) // pb
    pm = torch.zeros(nJ, B, device=dev)
    ps = torch.zeros(nJ, B, device=dev)
    pa = torch.zeros(nJ, B, dtype=torch.int32, device=dev)
    work = torch.empty(C().call("rg_head_work_bytes", B, HF), dtype=torch.uint8, device=dev)
    hd, Wd, bd = h.to(dev), W.to(dev), b.to(dev)
    for terms in (9, 6):
        C().call("rg_head_fwd_x", hd.data_ptr(), Wd.data_ptr(), bd.data_ptr(), B, A, HF, terms, None, 0,
                 pm.data_ptr(), ps.data_ptr(), pa.data_ptr(), 0, work.data_ptr(), st())
        work2 = torch.zeros(3 * min(128, nJ) * B, device=dev)
        amax = torch.zeros(B, dtype=torch.int32, device=dev)
        C().call("rg_lse_combine", pm.data_ptr(), ps.data_ptr(), pa.data_ptr(), B, nJ, work2.data_ptr(), None, 0,
                 None, A, None, amax.data_ptr(), None, None, st())
        zr = h.double() @ W.double().t() + b.double()
        zr[:, 1500], zr[:, 1999] = zr[:, 7], zr[:, 300]  # identical rows: exactly tied (BLAS edge tiles aside)
        ref = torch.argmax(zr, 1)
        assert set(ref.tolist()) <= {7, 300}
        assert torch.equal(amax.cpu().long(), ref)


def test_split_head_rejects_bad_shapes():
    dev = "cuda"
    x = torch.zeros(64, 128, device=dev)
    work = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    lib = C().load_library()
    # B not a multiple of 32; unknown term count
    assert lib.rg_head_fwd_x(x.data_ptr(), x.data_ptr(), x.data_ptr(), 40, 64, 128, 9, None, 0, x.data_ptr(),
                             x.data_ptr(), x.data_ptr(), 0, work.data_ptr(), st()) < 0
    assert lib.rg_head_fwd_x(x.data_ptr(), x.data_ptr(), x.data_ptr(), 64, 64, 128, 7, None, 0, x.data_ptr(),
                             x.data_ptr(), x.data_ptr(), 0, work.data_ptr(), st()) < 0
