"""Fused split-bf16 full-softmax training head (csrc/head_flash.hip) against
an fp64 torch restatement of the reference's nn.Linear + CrossEntropyLoss(mean)
forward / backward (GRU4Rec/model.py:58-60, 80, 121, 146): pass 1 (logits ->
online LSE -> unnormalised dh partials), the LSE / dh combine and pass 2 (dW,
db).  Kernel tolerances are those of the native fp32 path
(test_gpu_kernels.py::test_head_forward_backward); the trainer test holds the
north-star loss tolerance (1e-4) against the CPU oracle."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TERMS = {"f32x9": 9, "f32x6": 6, "f32x6d3": 636}
dev = "cuda"


def C():
    import recommenders.hip as h
    return h


def _u8(n):
    return torch.empty(int(n), dtype=torch.uint8, device=dev)


def run_flash(h, W, b, tgt, terms, nsplit, lo=0, lse_global=None, A_full=None, zs=False):
    """Every stage of the fused head through the C ABI; pass 2 in its
    gradient-only mode (dW_out / db_out).  zs: pass 1 stores the logits
    (rg_flash_fwd_top) and pass 2 reads them instead of recomputing S; the
    stored buffer is returned as "zs"."""
    call, st = C().call, C().stream_ptr()
    B, HF = h.shape
    A = W.shape[0]
    hb, wb = call("rg_head_plane_bytes", B, HF), call("rg_head_plane_bytes", A, HF)
    Hk, Hr, Wk, Wr = _u8(hb), _u8(hb), _u8(wb), _u8(wb)
    bp = torch.empty((A + 31) // 32 * 32, device=dev)
    call("rg_head_planes", h.data_ptr(), B, HF, Hk.data_ptr(), Hr.data_ptr(), None, None, st)
    call("rg_head_planes", W.data_ptr(), A, HF, Wk.data_ptr(), Wr.data_ptr(), b.data_ptr(), bp.data_ptr(), st)
    pm = torch.full((nsplit, B), float("nan"), device=dev)
    pl = torch.full((nsplit, B), float("nan"), device=dev)
    pO = torch.full((nsplit, HF, B), float("nan"), device=dev)
    zbuf = None
    if zs:
        zbuf = torch.full((call("rg_flash_zs_bytes", B, A) // 4,), float("nan"), device=dev)
        call("rg_flash_fwd_top", Hk.data_ptr(), Wk.data_ptr(), Wr.data_ptr(), bp.data_ptr(), B, A, HF, terms, nsplit,
             pm.data_ptr(), pl.data_ptr(), pO.data_ptr(), None, None, None, zbuf.data_ptr(), st)
    else:
        call("rg_flash_fwd", Hk.data_ptr(), Wk.data_ptr(), Wr.data_ptr(), bp.data_ptr(), B, A, HF, terms, nsplit,
             pm.data_ptr(), pl.data_ptr(), pO.data_ptr(), st)
    lse = torch.full((B,), float("nan"), device=dev)
    zt = torch.full((B,), float("nan"), device=dev)
    call("rg_flash_lse", pm.data_ptr(), pl.data_ptr(), nsplit, h.data_ptr(), W.data_ptr(), b.data_ptr(),
         tgt.data_ptr(), lo, A, lo + A if A_full is None else A_full, B, HF, lse.data_ptr(), zt.data_ptr(), st)
    rows = torch.empty(B, 2, device=dev)
    call("rg_flash_rows", (lse if lse_global is None else lse_global).data_ptr(), tgt.data_ptr(), lo, A, B,
         rows.data_ptr(), st)
    g = float(np.float32(1.0 / B))
    dh = torch.full((B, HF), float("nan"), device=dev)
    call("rg_flash_dh", pm.data_ptr(), pO.data_ptr(), rows.data_ptr(), nsplit, W.data_ptr(), g, B, HF,
         dh.data_ptr(), st)
    dW = torch.full((A, HF), float("nan"), device=dev)
    db = torch.full((A,), float("nan"), device=dev)
    if zs:
        call("rg_flash_dw_adam_planes", Hk.data_ptr(), Hr.data_ptr(), Wk.data_ptr(), bp.data_ptr(), rows.data_ptr(), g,
             B, A, HF, terms, None, None, None, None, None, None, None, dW.data_ptr(), db.data_ptr(), None, None, None,
             None, 0, zbuf.data_ptr(), st)
    else:
        call("rg_flash_dw_adam", Hk.data_ptr(), Hr.data_ptr(), Wk.data_ptr(), bp.data_ptr(), rows.data_ptr(), g, B, A,
             HF, terms, None, None, None, None, None, None, None, dW.data_ptr(), db.data_ptr(), st)
    torch.cuda.synchronize()
    out = {k: v.cpu().double() for k, v in dict(lse=lse, zt=zt, dh=dh, dW=dW, db=db).items()}
    if zs:
        out["zs"] = zbuf.cpu().double()
    return out


def zs_to_logits(zs, B, A):
    """(B, A) logits from the stored tiles (csrc/head_flash.hip k_flash_fwd: one
    1024-float tile per (32-item chunk, 32-row block), chunk-major; inside,
    quadrant (item half ib, row half rb), then 16-B slot 16a + 4(b >> 2) +
    ((b & 3) ^ a) holding the logits of items 16ib + 4a + u (u < 4), row
    16rb + b)."""
    nct = (A + 31) // 32
    t = zs.reshape(nct, B // 32, 2, 2, 64, 4)                # chunk, row block, ib, rb, slot, u
    a = torch.arange(4).view(4, 1)
    b = torch.arange(16).view(1, 16)
    slot = 16 * a + 4 * (b >> 2) + ((b & 3) ^ a)              # (a, b) -> slot
    t = t[:, :, :, :, slot.reshape(-1), :].reshape(nct, B // 32, 2, 2, 4, 16, 4)   # ..., a, b, u
    t = t.permute(1, 3, 5, 0, 2, 4, 6).reshape(B, nct * 32)   # row block, rb, b | chunk, ib, a, u
    return t[:, :A]


@pytest.mark.parametrize("B,A,HF", [(64, 1000, 32), (96, 3001, 64), (128, 4133, 128), (64, 2077, 256),
                                    (64, 20011, 64), (96, 40009, 128), (96, 78341, 64)])
def test_pass2_writes_next_planes(B, A, HF):
    """rg_flash_dw_adam_planes: the updated W / b leave as operand planes and
    padded bias bit-identical to rg_head_planes of the updated tensors (what
    the next pass 1 reads), incl. a ragged last item block; W / b / moments
    equal plain rg_flash_dw_adam's."""
    call, st = C().call, C().stream_ptr()
    h, W, b, tgt = inputs(B, A, HF, 3 + HF)
    h, W, b, tgt = h.to(dev), W.to(dev), b.to(dev), tgt.to(dev)
    hb, wb = call("rg_head_plane_bytes", B, HF), call("rg_head_plane_bytes", A, HF)
    Hk, Hr, Wk, Wr = _u8(hb), _u8(hb), _u8(wb), _u8(wb)
    bp = torch.empty((A + 31) // 32 * 32, device=dev)
    call("rg_head_planes", h.data_ptr(), B, HF, Hk.data_ptr(), Hr.data_ptr(), None, None, st)
    call("rg_head_planes", W.data_ptr(), A, HF, Wk.data_ptr(), Wr.data_ptr(), b.data_ptr(), bp.data_ptr(), st)
    ns = 8
    pm, pl, pO = torch.empty(ns, B, device=dev), torch.empty(ns, B, device=dev), torch.empty(ns, HF, B, device=dev)
    call("rg_flash_fwd", Hk.data_ptr(), Wk.data_ptr(), Wr.data_ptr(), bp.data_ptr(), B, A, HF, 6, ns, pm.data_ptr(),
         pl.data_ptr(), pO.data_ptr(), st)
    lse, zt, rows = torch.empty(B, device=dev), torch.empty(B, device=dev), torch.empty(B, 2, device=dev)
    call("rg_flash_lse", pm.data_ptr(), pl.data_ptr(), ns, h.data_ptr(), W.data_ptr(), b.data_ptr(), tgt.data_ptr(),
         0, A, A, B, HF, lse.data_ptr(), zt.data_ptr(), st)
    call("rg_flash_rows", lse.data_ptr(), tgt.data_ptr(), 0, A, B, rows.data_ptr(), st)
    adam6 = C().host_floats([0.1, 0.999, 0.001, 0.0316, 1e-8, -0.01])
    g = float(np.float32(1.0 / B))
    outs = []
    for planes in (False, True):
        Wx, bx = W.clone(), b.clone()
        mW, vW = torch.full_like(W, 0.01), torch.full_like(W, 0.02)
        mb, vb = torch.full_like(b, 0.01), torch.full_like(b, 0.02)
        Wk2, Wr2, bp2 = Wk.clone(), Wr.clone(), bp.clone()
        args = [Hk.data_ptr(), Hr.data_ptr(), Wk2.data_ptr(), bp2.data_ptr(), rows.data_ptr(), g, B, A, HF, 6,
                Wx.data_ptr(), mW.data_ptr(), vW.data_ptr(), bx.data_ptr(), mb.data_ptr(), vb.data_ptr(), adam6,
                None, None]
        if planes:
            nb = call("rg_flash_dw_work_bytes", B, A, HF)
            work = _u8(max(nb, 16))
            call("rg_flash_dw_adam_planes", *args, Wk2.data_ptr(), Wr2.data_ptr(), bp2.data_ptr(), work.data_ptr(),
                 nb, None, st)
        else:
            call("rg_flash_dw_adam", *args, st)
        torch.cuda.synchronize()
        outs.append((Wx, bx, mW, vW, mb, vb, Wk2, Wr2, bp2))
    for x, y in zip(outs[0][:6], outs[1][:6]):   # (the tail split sums in another order: allclose)
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)
    Wx, bx = outs[1][0], outs[1][1]
    Wk3, Wr3, bp3 = _u8(wb), _u8(wb), torch.empty_like(bp)
    call("rg_head_planes", Wx.data_ptr(), A, HF, Wk3.data_ptr(), Wr3.data_ptr(), bx.data_ptr(), bp3.data_ptr(), st)
    torch.cuda.synchronize()
    assert not torch.equal(Wk3, Wk)   # W moved
    assert torch.equal(outs[1][6], Wk3)
    assert torch.equal(outs[1][7], Wr3)
    assert torch.equal(outs[1][8], bp3)


@pytest.mark.parametrize("B,A,HF", [(96, 78341, 64), (128, 78341, 64), (64, 70000, 128)])
def test_pass2_tail_split_matches_fp64(B, A, HF):
    """Pass 2 with its leftover item blocks split over the row chunks
    (rg_flash_dw_adam_planes with work; 306 blocks of 256 = 256 whole + 50
    split 3 / 4 ways, HF 64; 274 = 256 + 18 at HF 128): raw dW / db against
    fp64 at the fused head's tolerances, and nonzero split work."""
    call, st = C().call, C().stream_ptr()
    nb = call("rg_flash_dw_work_bytes", B, A, HF)
    assert nb > 0
    h, W, b, tgt = inputs(B, A, HF, 17)
    r = fp64_reference(h, W, b, tgt)
    h, W, b, tgt = h.to(dev), W.to(dev), b.to(dev), tgt.to(dev)
    o = run_flash(h, W, b, tgt, 6, 8)   # dh, lse via the plain path (no tail split)
    hb, wb = call("rg_head_plane_bytes", B, HF), call("rg_head_plane_bytes", A, HF)
    Hk, Hr, Wk, Wr = _u8(hb), _u8(hb), _u8(wb), _u8(wb)
    bp = torch.empty((A + 31) // 32 * 32, device=dev)
    call("rg_head_planes", h.data_ptr(), B, HF, Hk.data_ptr(), Hr.data_ptr(), None, None, st)
    call("rg_head_planes", W.data_ptr(), A, HF, Wk.data_ptr(), Wr.data_ptr(), b.data_ptr(), bp.data_ptr(), st)
    rows = torch.empty(B, 2, device=dev)
    call("rg_flash_rows", o["lse"].float().to(dev).data_ptr(), tgt.data_ptr(), 0, A, B, rows.data_ptr(), st)
    dW = torch.full((A, HF), float("nan"), device=dev)
    db = torch.full((A,), float("nan"), device=dev)
    work = _u8(nb)
    g = float(np.float32(1.0 / B))
    call("rg_flash_dw_adam_planes", Hk.data_ptr(), Hr.data_ptr(), Wk.data_ptr(), bp.data_ptr(), rows.data_ptr(), g, B,
         A, HF, 6, None, None, None, None, None, None, None, dW.data_ptr(), db.data_ptr(), None, None, None,
         work.data_ptr(), nb, None, st)
    torch.cuda.synchronize()
    torch.testing.assert_close(dW.cpu().double(), r["dW"], rtol=0, atol=1e-7)
    torch.testing.assert_close(db.cpu().double(), r["db"], rtol=0, atol=1e-7)


def fp64_reference(h, W, b, tgt):
    Wr = W.double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    hr = h.double().requires_grad_(True)
    Z = hr @ Wr.t() + br
    torch.nn.functional.cross_entropy(Z, tgt).backward()
    Z = Z.detach()
    return dict(Z=Z, lse=torch.logsumexp(Z, 1), zt=Z.gather(1, tgt[:, None])[:, 0], dh=hr.grad, dW=Wr.grad,
                db=br.grad)


def inputs(B, A, HF, seed):
    g = torch.Generator().manual_seed(seed)
    h = torch.randn(B, HF, generator=g) * 0.5
    W = torch.randn(A, HF, generator=g) * 0.1
    b = torch.randn(A, generator=g) * 0.1
    tgt = torch.randint(0, A, (B,), generator=g)
    return h, W, b, tgt


# (B, A, HF, nsplit): partial 256-row (HF 256: 128-row) workgroups, ragged last item
# chunk (A % 32 != 0), empty splits (512 × 2077 with 64 splits), split counts
# with and without the XCD reorder (total workgroups % 8)
@pytest.mark.parametrize("precision", ["f32x9", "f32x6", "f32x6d3"])
@pytest.mark.parametrize("B,A,HF,nsplit", [(64, 1000, 32, 8), (128, 3001, 64, 16), (256, 4133, 128, 8),
                                           (512, 2077, 128, 64), (96, 777, 128, 3), (288, 50000, 128, 16),
                                           (256, 3001, 256, 8), (96, 2077, 256, 24), (160, 777, 256, 3)])
def test_flash_head_matches_fp64(precision, B, A, HF, nsplit):
    h, W, b, tgt = inputs(B, A, HF, B + A + HF)
    o = run_flash(h.to(dev), W.to(dev), b.to(dev), tgt.to(dev), TERMS[precision], nsplit)
    r = fp64_reference(h, W, b, tgt)
    torch.testing.assert_close(o["lse"], r["lse"], rtol=0, atol=2e-5)
    torch.testing.assert_close(o["lse"] - o["zt"], r["lse"] - r["zt"], rtol=0, atol=2e-5)  # per-row CE
    torch.testing.assert_close(o["dh"], r["dh"], rtol=0, atol=1e-6)
    torch.testing.assert_close(o["dW"], r["dW"], rtol=0, atol=1e-7)
    torch.testing.assert_close(o["db"], r["db"], rtol=0, atol=1e-7)


@pytest.mark.parametrize("precision", ["f32x6", "f32x6d3"])
@pytest.mark.parametrize("B,A,HF,nsplit", [(256, 1000, 32, 8), (256, 3001, 64, 16), (256, 4133, 128, 8),
                                           (512, 2077, 128, 64), (768, 777, 128, 3), (512, 50000, 128, 16),
                                           (256, 3001, 256, 8), (128, 2077, 256, 24), (384, 777, 256, 3),
                                           (512, 30011, 256, 16)])
def test_stored_logits_match_fp64(precision, B, A, HF, nsplit):
    """Stored-logit head (zs): pass 1 writes z = h·Wᵀ + b tile by tile, pass 2
    reads it instead of recomputing the S contraction.  The stored logits
    against fp64 (and −inf past A inside the last chunk), and every output at
    the recomputing head's tolerances; dW / db within a few fp32 ulps of the
    recomputing pass 2's (same products, other accumulation order)."""
    h, W, b, tgt = inputs(B, A, HF, B + A + HF)
    hd, Wd, bd, td = h.to(dev), W.to(dev), b.to(dev), tgt.to(dev)
    o = run_flash(hd, Wd, bd, td, TERMS[precision], nsplit, zs=True)
    o2 = run_flash(hd, Wd, bd, td, TERMS[precision], nsplit)
    r = fp64_reference(h, W, b, tgt)
    nct = (A + 31) // 32
    Z = zs_to_logits(o["zs"], B, nct * 32)
    # (fp32 accumulation of HF split-bf16 products: the bound grows with HF)
    torch.testing.assert_close(Z[:, :A], r["Z"], rtol=0, atol=2e-6 * max(1, HF // 128))
    assert torch.isneginf(Z[:, A:]).all()
    torch.testing.assert_close(o["lse"], r["lse"], rtol=0, atol=2e-5)
    torch.testing.assert_close(o["dh"], r["dh"], rtol=0, atol=1e-6)
    torch.testing.assert_close(o["dW"], r["dW"], rtol=0, atol=1e-7)
    torch.testing.assert_close(o["db"], r["db"], rtol=0, atol=1e-7)
    torch.testing.assert_close(o["dW"], o2["dW"], rtol=0, atol=2e-8)
    torch.testing.assert_close(o["db"], o2["db"], rtol=0, atol=2e-8)


@pytest.mark.parametrize("B,HF", [(192, 256), (96, 64), (288, 128)])
def test_stored_logits_refused_shapes(B, HF):
    """Stored logits need whole pass-1 row blocks (256 rows; 128 at HF 256):
    the trainers then recompute in pass 2."""
    call = C().call
    A = 1000
    z = torch.empty(call("rg_flash_zs_bytes", B, A) // 4, device=dev)
    x = torch.empty(16, device=dev)
    with pytest.raises(RuntimeError, match="status -3"):   # RG_ERR_SHAPE, nothing launched
        call("rg_flash_fwd_top", x.data_ptr(), x.data_ptr(), x.data_ptr(), x.data_ptr(), B, A, HF, 6, 8, x.data_ptr(),
             x.data_ptr(), x.data_ptr(), None, None, None, z.data_ptr(), C().stream_ptr())


@pytest.mark.parametrize("B,A,HF,K", [(256, 20011, 128, 1), (256, 20011, 128, 5), (128, 5003, 256, 1),
                                       (256, 5003, 256, 12)])
def test_stored_logit_pass1_top_entries_unchanged(B, A, HF, K):
    """The SMORL trainers' pass 1 stores the logits while emitting the
    rewards' top-k inputs (per-split first maxima, chunk maxima): the top-k
    lists and values equal those of the same pass without the stores, bit
    for bit (HF 256 stores from inside the softmax section)."""
    h, W, b, tgt = inputs(B, A, HF, 11 + K)
    hd, Wd, bd = h.to(dev), W.to(dev), b.to(dev)
    i1, v1, e1, c1 = run_top(hd, Wd, bd, 636, 8, K, exact1=True, zs=True)
    i0, v0, e0, c0 = run_top(hd, Wd, bd, 636, 8, K, exact1=True)
    assert torch.equal(i1, i0) and torch.equal(v1, v0) and e1 == e0
    assert torch.equal(c1, c0)


@pytest.mark.parametrize("B,A,HF", [(256, 78341, 64), (512, 70000, 128), (256, 40011, 256)])
def test_stored_logits_tail_split_adam(B, A, HF):
    """Stored logits through the trainer's pass 2 (Adam + next planes, the
    leftover item blocks split over the row chunks): W / b / moments and the
    planes equal the recomputing pass 2's within fp32 rounding."""
    call, st = C().call, C().stream_ptr()
    h, W, b, tgt = inputs(B, A, HF, 5 + HF)
    h, W, b, tgt = h.to(dev), W.to(dev), b.to(dev), tgt.to(dev)
    hb, wb = call("rg_head_plane_bytes", B, HF), call("rg_head_plane_bytes", A, HF)
    Hk, Hr, Wk, Wr = _u8(hb), _u8(hb), _u8(wb), _u8(wb)
    bp = torch.empty((A + 31) // 32 * 32, device=dev)
    call("rg_head_planes", h.data_ptr(), B, HF, Hk.data_ptr(), Hr.data_ptr(), None, None, st)
    call("rg_head_planes", W.data_ptr(), A, HF, Wk.data_ptr(), Wr.data_ptr(), b.data_ptr(), bp.data_ptr(), st)
    ns = 8
    pm, pl, pO = torch.empty(ns, B, device=dev), torch.empty(ns, B, device=dev), torch.empty(ns, HF, B, device=dev)
    zbuf = torch.empty(call("rg_flash_zs_bytes", B, A) // 4, device=dev)
    call("rg_flash_fwd_top", Hk.data_ptr(), Wk.data_ptr(), Wr.data_ptr(), bp.data_ptr(), B, A, HF, 636, ns,
         pm.data_ptr(), pl.data_ptr(), pO.data_ptr(), None, None, None, zbuf.data_ptr(), st)
    lse, zt, rows = torch.empty(B, device=dev), torch.empty(B, device=dev), torch.empty(B, 2, device=dev)
    call("rg_flash_lse", pm.data_ptr(), pl.data_ptr(), ns, h.data_ptr(), W.data_ptr(), b.data_ptr(), tgt.data_ptr(),
         0, A, A, B, HF, lse.data_ptr(), zt.data_ptr(), st)
    call("rg_flash_rows", lse.data_ptr(), tgt.data_ptr(), 0, A, B, rows.data_ptr(), st)
    adam6 = C().host_floats([0.1, 0.999, 0.001, 0.0316, 1e-8, -0.01])
    g = float(np.float32(1.0 / B))
    nb = call("rg_flash_dw_work_bytes", B, A, HF)
    assert nb > 0
    outs = []
    for use_z in (False, True):
        Wx, bx = W.clone(), b.clone()
        mW, vW = torch.full_like(W, 0.01), torch.full_like(W, 0.02)
        mb, vb = torch.full_like(b, 0.01), torch.full_like(b, 0.02)
        Wk2, Wr2, bp2 = Wk.clone(), Wr.clone(), bp.clone()
        work = _u8(nb)
        call("rg_flash_dw_adam_planes", Hk.data_ptr(), Hr.data_ptr(), Wk2.data_ptr(), bp2.data_ptr(), rows.data_ptr(),
             g, B, A, HF, 636, Wx.data_ptr(), mW.data_ptr(), vW.data_ptr(), bx.data_ptr(), mb.data_ptr(),
             vb.data_ptr(), adam6, None, None, Wk2.data_ptr(), Wr2.data_ptr(), bp2.data_ptr(), work.data_ptr(), nb,
             zbuf.data_ptr() if use_z else None, st)
        torch.cuda.synchronize()
        outs.append((Wx, bx, mW, vW, mb, vb))
    for x, y in zip(outs[0], outs[1]):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-7)


def test_flash_head_item_shard():
    """One rank's item shard [lo, hi): local lse and owner-only target logit;
    the backward with the all-rank lse gives the shard's part of dh and its
    rows of dW / db (recommenders/hip/sharded.py)."""
    B, A, HF = 128, 5000, 64
    lo, hi = 1800, 3900
    h, W, b, tgt = inputs(B, A, HF, 77)
    r = fp64_reference(h, W, b, tgt)
    o = run_flash(h.to(dev), W[lo:hi].contiguous().to(dev), b[lo:hi].contiguous().to(dev), tgt.to(dev), 6, 8,
                  lo=lo, lse_global=r["lse"].float().to(dev), A_full=A)
    torch.testing.assert_close(o["lse"], torch.logsumexp(r["Z"][:, lo:hi], 1), rtol=0, atol=2e-5)
    own = (tgt >= lo) & (tgt < hi)
    assert 0 < int(own.sum()) < B
    torch.testing.assert_close(o["zt"], torch.where(own, r["zt"], torch.zeros_like(r["zt"])), rtol=0, atol=1e-5)
    P = torch.softmax(r["Z"], 1)
    P[torch.arange(B), tgt] -= 1.0
    P /= B
    torch.testing.assert_close(o["dh"], P[:, lo:hi] @ W[lo:hi].double(), rtol=0, atol=1e-6)
    torch.testing.assert_close(o["dW"], r["dW"][lo:hi], rtol=0, atol=1e-7)
    torch.testing.assert_close(o["db"], r["db"][lo:hi], rtol=0, atol=1e-7)


@pytest.mark.parametrize("precision", ["f32x6", "f32x9", "f32x6d3"])
def test_flash_invalid_target_gives_nan_row(precision):
    """A target outside [0, A) gives a NaN loss row on the fused head, as on
    the native head (CrossEntropyLoss raises there); the trainer's loss is NaN."""
    B, A, HF = 64, 3000, 64
    h, W, b, tgt = inputs(B, A, HF, 11)
    tgt[3], tgt[17] = A, -1
    o = run_flash(h.to(dev), W.to(dev), b.to(dev), tgt.to(dev), TERMS[precision], 8)
    ce = o["lse"] - o["zt"]
    assert torch.isnan(ce[3]) and torch.isnan(ce[17])
    ok = torch.ones(B, dtype=torch.bool)
    ok[[3, 17]] = False
    assert torch.isfinite(ce[ok]).all()
    from recommenders.data_utils.synthetic import SessionStream
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
    tr = GRU4Rec_trainer(hidden_dim=32, embedding_dim=32, gru_layers=1, train_pad_embed=True, use_packed_seq=True,
                         learning_rate=0.01, item_num=500, state_size=6, action_dim=500, device="cuda",
                         matmul_precision=precision)
    s, a, r, sn, ln, nln, e = SessionStream(500, 6, 64, seed=3).batch(0, 64)
    a[5] = 500
    assert np.isnan(tr.train_step(s, a, ln))


@pytest.mark.parametrize("precision", ["f32x9", "f32x6", "f32x6d3"])
def test_flash_trainer_matches_oracle(precision):
    """GRU4Rec with the full softmax at C2 widths (H 128, L 50), scaled down, on
    the fused head: same loss / weight tolerances as the native path
    (test_gpu_supervised.py::test_gru4rec_matches_oracle_medium)."""
    from oracle.models import OracleSupervised
    from recommenders.data_utils.synthetic import SessionStream
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
    E = H = 128
    N, L, B = 50000, 50, 1024
    cfg = dict(hidden_dim=H, embedding_dim=E, gru_layers=1, train_pad_embed=True, use_packed_seq=True,
               learning_rate=0.005, item_num=N, state_size=L, action_dim=N)
    torch.set_num_threads(8)
    orc = OracleSupervised(kind="gru4rec", **cfg)
    tr = GRU4Rec_trainer(device="cuda", matmul_precision=precision, **cfg)
    assert tr.gru_model.heads["output"].flash_terms(B) == TERMS[precision]
    st = SessionStream(N, L, B * 3, seed=9)
    for i in range(3):
        s, a, r, sn, ln, nln, e = st.batch(i, B)
        lo = orc.step(s, a, ln)
        lg = tr.train_step(s, a, ln)
        assert abs(lo - lg) < 1e-4, (i, lo, lg)
    assert tr.gru_model.heads["output"].stored_logits()   # B 1024, HF 128: the stored-logit head ran
    sd_o = orc.net.state_dict()
    for k, v in tr.gru_model.state_dict().items():
        d = (v.cpu() - sd_o[k]).abs()
        assert float(d.max()) <= 2 * cfg["learning_rate"] + 1e-5, k
        assert float((d > 1e-4).float().mean()) < 1e-3, (k, float((d > 1e-4).float().mean()))


@pytest.mark.parametrize("kind,E", [("gru4rec", 64), ("smorl", 64), ("smorl", 256)])
def test_stored_logit_trainer_equals_recomputing(kind, E):
    """The trainers with stored logits (default where they fit) and with
    pass 2 recomputing them (head.zstore = False) take the same steps (same
    plane products, other accumulation order): losses within 1e-5, weights at
    the training tolerances of the oracle tests (Adam's normalised step can
    turn a last-bit difference of a near-zero gradient into up to 2·lr) —
    GRU4Rec, and SMORL's supervised head (pass 1 with the top-k outputs and the
    stored logits together; E 256: the C5 width, HF 256 stores from the
    softmax section, 128-row blocks)."""
    import random
    from recommenders.data_utils.synthetic import SessionStream
    N, L, B = 20000, 12, 512
    cfg = dict(hidden_dim=E, embedding_dim=E, gru_layers=1, train_pad_embed=True, use_packed_seq=True,
               learning_rate=0.005, item_num=N, state_size=L, action_dim=N)
    st = SessionStream(N, L, B * 3, seed=13)
    runs = []
    for zstore in (None, False):
        random.seed(3)
        if kind == "gru4rec":
            from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
            tr = GRU4Rec_trainer(device="cuda", **cfg)
            nets, heads = (tr.gru_model,), [tr.gru_model.heads["output"]]
        else:
            from recommenders.models.SMORL.smorl_gru import SMORL_trainer
            g = torch.Generator().manual_seed(7)
            tr = SMORL_trainer(device="cuda", padding_pos="end", gamma=0.5, q_weights=[1.0, 0.5, 2.0], alpha=1.0,
                               div_embedding=torch.randn(N + 1, 16, generator=g) * 0.01,
                               unpopular_actions_set=set(range(0, N, 3)), topk_div=2, topk_nov=1, **cfg)
            nets = (tr.SMORL_1, tr.SMORL_2)
            heads = [n.sup_head_output for n in nets]
        for hd in heads:
            hd.zstore = zstore
        losses = []
        for i in range(3):
            b = st.batch(i, B)
            out = tr.train_step(b[0], b[1], b[4]) if kind == "gru4rec" else tr.train_step(*b)
            losses.append(np.atleast_1d(np.array(out, dtype=np.float64)))
        assert any(hd.stored_logits() for hd in heads) == (zstore is None)
        runs.append((np.concatenate(losses), [{k: v.cpu() for k, v in n.state_dict().items()} for n in nets]))
    np.testing.assert_allclose(runs[0][0], runs[1][0], rtol=0, atol=1e-5)
    lr = cfg["learning_rate"]
    for sd0, sd1 in zip(runs[0][1], runs[1][1]):
        for k in sd0:
            d = (sd0[k] - sd1[k]).abs()
            assert float(d.max()) <= 2 * lr + 1e-5, k
            assert float((d > 1e-4).float().mean()) < 1e-3, (k, float((d > 1e-4).float().mean()))


def run_native(h, W, b, tgt):
    """The native fp32-MFMA path (csrc/head.hip: Zᵀ stored, dh / dW from it)."""
    call, st = C().call, C().stream_ptr()
    B, HF = h.shape
    A = W.shape[0]
    ldz = (B + 3) // 4 * 4
    nJ = (A + C().load_library().rg_partial_block() - 1) // C().load_library().rg_partial_block()
    ZT = torch.zeros(A, ldz, device=dev)
    pm, ps = torch.zeros(nJ, B, device=dev), torch.zeros(nJ, B, device=dev)
    pa = torch.zeros(nJ, B, dtype=torch.int32, device=dev)
    call("rg_head_fwd", h.data_ptr(), W.data_ptr(), b.data_ptr(), B, A, HF, ZT.data_ptr(), ldz, pm.data_ptr(),
         ps.data_ptr(), pa.data_ptr(), 1, st)
    work = torch.zeros(3 * min(128, nJ) * B, device=dev)
    lse = torch.zeros(B, device=dev)
    lrow = torch.zeros(B, device=dev)
    call("rg_lse_combine", pm.data_ptr(), ps.data_ptr(), pa.data_ptr(), B, nJ, work.data_ptr(), ZT.data_ptr(), ldz,
         tgt.data_ptr(), A, lse.data_ptr(), None, lrow.data_ptr(), None, st)
    g = float(np.float32(1.0 / B))
    slabs = torch.zeros(8, B, HF, device=dev)
    n = call("rg_head_dh", ZT.data_ptr(), ldz, lse.data_ptr(), tgt.data_ptr(), g, W.data_ptr(), B, A, HF, 8,
             slabs.data_ptr(), st)
    dW = torch.zeros(A, HF, device=dev)
    db = torch.zeros(A, device=dev)
    call("rg_head_dw_adam", ZT.data_ptr(), ldz, lse.data_ptr(), tgt.data_ptr(), g, h.data_ptr(), B, A, HF,
         None, None, None, None, None, None, None, dW.data_ptr(), db.data_ptr(), st)
    torch.cuda.synchronize()
    return {k: v.cpu().double() for k, v in dict(lse=lse, ce=lrow, dh=slabs[:n].sum(0), dW=dW, db=db).items()}


# max |error| against fp64 of the reference's own CPU fp32 path (torch CPU,
# tools/prec_err.py's cases 1-3; measured in this container): the split
# precisions are also held to a small multiple of it
CPU_F32_ERR = [dict(lse=9.509e-07, ce=1.030e-06, dh=9.857e-10, dW=1.671e-09, db=4.977e-10),
               dict(lse=1.088e-05, ce=1.079e-05, dh=1.677e-08, dW=8.981e-09, db=9.728e-09),
               dict(lse=9.957e-07, ce=2.708e-06, dh=1.818e-09, dW=1.552e-09, db=1.446e-09)]
ERR_CASES = [(512, 30000, 128, 0.5, 0.1, 5), (512, 30000, 128, 0.9, 0.6, 6), (1024, 100000, 128, 0.9, 0.3, 7)]


@pytest.mark.parametrize("case", [0, 1, 2])
def test_flash_error_is_fp32_class(case):
    """Max |error| against fp64 of the fused split head next to the native
    fp32-MFMA path on the same inputs (lse, per-row CE, dh, dW, db): within 4×
    of native and 2× of the reference's CPU fp32 path for f32x9, f32x6 and
    f32x6d3 (floor: 8 fp32 ulps of the quantity's scale).  Case 1 has logits
    up to 26 (trained-like scale); f32x6d3's dh (O at 3 plane products) is
    the only output that differs from f32x6."""
    B, A, HF, hs, ws, seed = ERR_CASES[case]
    g = torch.Generator().manual_seed(seed)
    h = torch.tanh(torch.randn(B, HF, generator=g) * 2) * hs
    W = torch.randn(A, HF, generator=g) * ws
    b = torch.randn(A, generator=g) * ws
    tgt = torch.randint(0, A, (B,), generator=g)
    r = fp64_reference(h, W, b, tgt)
    r["ce"] = r["lse"] - r["zt"]
    hd, Wd, bd, td = h.to(dev), W.to(dev), b.to(dev), tgt.to(dev)
    errs = {"f32": run_native(hd, Wd, bd, td)}
    for p in TERMS:
        o = run_flash(hd, Wd, bd, td, TERMS[p], 16)
        o["ce"] = o["lse"] - o["zt"]
        errs[p] = o
    keys = ("lse", "ce", "dh", "dW", "db")
    table = {p: {k: float((o[k] - r[k]).abs().max()) for k in keys} for p, o in errs.items()}
    print(table)
    for k in keys:
        floor = 8 * 2.0 ** -24 * float(r[k].abs().max())
        for p in TERMS:
            assert table[p][k] <= max(4 * table["f32"][k], floor), (p, k, table)
            assert table[p][k] <= max(2 * CPU_F32_ERR[case][k], floor), (p, k, table)
    for k in ("lse", "ce", "dW", "db"):   # f32x6d3 changes only the dh contraction
        assert table["f32x6d3"][k] == table["f32x6"][k], (k, table)


# ------------------------------------------------------------- fused top-k --
def run_top(h, W, b, terms, nsplit, K, exact1=False, zs=False):
    """Pass 1 with the top-k outputs, then rg_flash_argmax (K = 1, unless
    exact1: the trainers' K = 1 re-scoring) or rg_flash_topk:
    (idx (B, K) int64, vals (B, K) f64, err).  zs: pass 1 also stores the
    logits (the SMORL trainers' stored-logit pass 1)."""
    call, st = C().call, C().stream_ptr()
    B, HF = h.shape
    A = W.shape[0]
    hb, wb = call("rg_head_plane_bytes", B, HF), call("rg_head_plane_bytes", A, HF)
    Hk, Hr, Wk, Wr = _u8(hb), _u8(hb), _u8(wb), _u8(wb)
    bp = torch.empty((A + 31) // 32 * 32, device=dev)
    call("rg_head_planes", h.data_ptr(), B, HF, Hk.data_ptr(), Hr.data_ptr(), None, None, st)
    call("rg_head_planes", W.data_ptr(), A, HF, Wk.data_ptr(), Wr.data_ptr(), b.data_ptr(), bp.data_ptr(), st)
    z = lambda *s, dt=torch.float32: torch.full(s, -7, dtype=dt, device=dev)  # noqa: E731
    pm, pl, pO = z(nsplit, B), z(nsplit, B), z(nsplit, HF, B)
    pbest, parg = z(nsplit, B), z(nsplit, B, dt=torch.int32)
    cmax = z((A + 31) // 32, B) if K > 1 or exact1 else None
    zbuf = torch.empty(call("rg_flash_zs_bytes", B, A) // 4, device=dev) if zs else None
    call("rg_flash_fwd_top", Hk.data_ptr(), Wk.data_ptr(), Wr.data_ptr(), bp.data_ptr(), B, A, HF, terms, nsplit,
         pm.data_ptr(), pl.data_ptr(), pO.data_ptr(), pbest.data_ptr(), parg.data_ptr(),
         None if cmax is None else cmax.data_ptr(), None if zbuf is None else zbuf.data_ptr(), st)
    idx, vals = z(B, K, dt=torch.int32), z(B, K)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    if K == 1 and not exact1:
        call("rg_flash_argmax", pbest.data_ptr(), parg.data_ptr(), nsplit, B, idx.data_ptr(), vals.data_ptr(), st)
    else:
        cap = call("rg_flash_topk_cap")
        cand, ncand = z(B, cap, dt=torch.int32), z(B, dt=torch.int32)
        work = _u8(call("rg_flash_topk_work_bytes", B, A, K))
        call("rg_flash_topk", cmax.data_ptr(), B, B, A, K, 1e-4, 1e-4, h.data_ptr(), W.data_ptr(), b.data_ptr(), HF,
             cand.data_ptr(), ncand.data_ptr(), idx.data_ptr(), vals.data_ptr(), err.data_ptr(), work.data_ptr(), st)
    torch.cuda.synchronize()
    return idx.cpu().long(), vals.cpu().double(), int(err.item()), (None if cmax is None else cmax.cpu().double())


@pytest.mark.parametrize("precision", ["f32x6", "f32x9", "f32x6d3"])
@pytest.mark.parametrize("B,A,HF,nsplit,K", [(128, 3001, 64, 8, 1), (96, 20011, 128, 16, 1), (256, 5000, 256, 8, 1),
                                             (128, 3001, 64, 8, 12), (96, 20011, 128, 16, 20),
                                             (160, 5003, 256, 8, 12), (64, 777, 32, 3, 32)])
def test_fused_topk_matches_canonical_fp64(precision, B, A, HF, nsplit, K):
    """torch.topk(sup, K) of SMORL's rewards (diversity.py:15-73, novelty.py:12-47)
    from pass 1 without logits: index lists equal the canonical (value desc,
    index asc) top-K of the fp64 logits except where two logits lie within the
    arithmetic's error bound; values within fp32 rounding of fp64; chunk maxima
    exact to the split-bf16 bound."""
    from oracle import metrics as om
    h, W, b, _ = inputs(B, A, HF, 3 * B + A + K)
    idx, vals, err, cmax = run_top(h.to(dev), W.to(dev), b.to(dev), TERMS[precision], nsplit, K)
    assert err == 0
    Z = (h.double() @ W.double().t() + b.double()).numpy()
    ref = om.canonical_topk_fast(Z, K)
    got = idx.numpy()
    tol = 2e-5
    flips, gap = om.topk_flip_report(Z, got, ref, tol)
    assert flips <= max(1, B // 50), (flips, gap)
    np.testing.assert_allclose(vals.numpy(), np.take_along_axis(Z, got, 1), rtol=0, atol=tol)
    # the device list is canonical in its own values
    v = vals.numpy()
    assert ((v[:, :-1] > v[:, 1:]) | ((v[:, :-1] == v[:, 1:]) & (got[:, :-1] < got[:, 1:]))).all()
    if cmax is not None:
        nct = (A + 31) // 32
        Zp = np.full((B, nct * 32), -np.inf)
        Zp[:, :A] = Z
        np.testing.assert_allclose(cmax.numpy().T, Zp.reshape(B, nct, 32).max(2), rtol=0, atol=tol)


@pytest.mark.parametrize("precision", ["f32x6", "f32x6d3"])
@pytest.mark.parametrize("B,A,HF,nsplit", [(128, 50000, 128, 16), (64, 5003, 256, 8), (96, 3001, 64, 8)])
def test_fused_top1_rescored_is_first_fp32_maximum(precision, B, A, HF, nsplit):
    """SMORL's top-1 reward item (topk_div = topk_nov = 1, the C4 bench
    setting) through the trainers' path: pass 1's chunk maxima + rg_flash_topk
    with K = 1, i.e. the fp32 re-scoring — the first maximum of the fp32
    logits also where the split-bf16 logits alone could pick another item:
    planted exact duplicates (lowest index wins) and near-ties 1e-6 apart."""
    h, W, b, _ = inputs(B, A, HF, 5 * B + A)
    Z = h.double() @ W.double().t() + b.double()
    top = Z.argmax(1)
    for r in range(0, B, 3):            # exact tie: a copy of the winner at a higher index
        j = int(top[r])
        k = (j * 7919 + 13) % A
        if k > j:
            W[k], b[k] = W[j], b[j]
    for r in range(1, B, 3):            # near tie: a slightly better copy at a lower index
        j = int(top[r])
        k = (j * 104729 + 7) % A
        if k < j:
            W[k], b[k] = W[j], b[j] + 1e-6
    Z = h.double() @ W.double().t() + b.double()
    idx, vals, err, _ = run_top(h.to(dev), W.to(dev), b.to(dev), TERMS[precision], nsplit, 1, exact1=True)
    assert err == 0
    zmax = Z.max(1).values
    first = (Z >= zmax[:, None]).double().argmax(1)
    sl = (h.abs().double() @ W.abs().double().t()).max(1).values
    for r in range(B):
        if int(idx[r, 0]) != int(first[r]):
            assert float(zmax[r] - Z[r, idx[r, 0]]) <= 200 * 2.0 ** -24 * float(sl[r]), r
    for r in range(0, B, 3):
        assert int(idx[r, 0]) == int(first[r])
    for r in range(1, B, 3):
        assert int(idx[r, 0]) == int(first[r])


def test_fused_topk_exact_ties_keep_lowest_index():
    """Exact ties (duplicated W rows and biases): lowest item first, as the
    canonical order and torch.argmax's first maximum."""
    B, A, HF, K = 64, 4000, 64, 5
    h, W, b, _ = inputs(B, A, HF, 21)
    for j, src in ((3999, 17), (2500, 17), (1234, 17), (60, 800)):
        W[j], b[j] = W[src], b[src]
    # make item 17 every row's maximum
    b[17] = b[3999] = b[2500] = b[1234] = 50.0
    for K_ in (1, K):
        idx, vals, err, _ = run_top(h.to(dev), W.to(dev), b.to(dev), 6, 8, K_)
        assert err == 0
        assert (idx[:, 0] == 17).all()
        if K_ > 1:
            assert (idx[:, 1:4] == torch.tensor([1234, 2500, 3999])).all()


@pytest.mark.parametrize("precision", ["f32x6", "f32x9", "f32x6d3"])
@pytest.mark.parametrize("B,A,HF,nsplit", [(128, 3001, 64, 8), (96, 20011, 128, 16), (160, 5003, 256, 8),
                                           (64, 777, 32, 3)])
def test_fused_argmax_only(precision, B, A, HF, nsplit):
    """rg_flash_amax_fwd (the double-Q target's argmax on split-bf16 MFMAs,
    sqn_gru.py:222-226): the first maximum of the fp64 logits except where the
    top two lie within the arithmetic's error bound; the returned maxima
    within fp32 rounding; exact duplicates resolve to the lowest index."""
    call, st = C().call, C().stream_ptr()
    h, W, b, _ = inputs(B, A, HF, 7 * B + A)
    W[A - 5], b[A - 5] = W[11], b[11]          # an exact duplicate of item 11 later in the table
    hd, Wd, bd = h.to(dev), W.to(dev), b.to(dev)
    Hk, Wk = _u8(call("rg_head_plane_bytes", B, HF)), _u8(call("rg_head_plane_bytes", A, HF))
    bp = torch.empty((A + 31) // 32 * 32, device=dev)
    call("rg_head_planes", hd.data_ptr(), B, HF, Hk.data_ptr(), None, None, None, st)
    call("rg_head_planes", Wd.data_ptr(), A, HF, Wk.data_ptr(), None, bd.data_ptr(), bp.data_ptr(), st)
    pbest = torch.full((nsplit, B), -7.0, device=dev)
    parg = torch.full((nsplit, B), -7, dtype=torch.int32, device=dev)
    call("rg_flash_amax_fwd", Hk.data_ptr(), Wk.data_ptr(), bp.data_ptr(), B, A, HF, TERMS[precision], nsplit,
         pbest.data_ptr(), parg.data_ptr(), st)
    idx = torch.empty(B, dtype=torch.int32, device=dev)
    mx = torch.empty(B, device=dev)
    call("rg_flash_argmax", pbest.data_ptr(), parg.data_ptr(), nsplit, B, idx.data_ptr(), mx.data_ptr(), st)
    torch.cuda.synchronize()
    Z = (h.double() @ W.double().t() + b.double()).numpy()
    got = idx.cpu().long().numpy()
    ref = Z.argmax(1)
    gap = np.abs(Z[np.arange(B), got] - Z[np.arange(B), ref])
    assert (gap[got != ref] < 2e-5).all()
    assert (got != ref).sum() <= max(1, B // 50)
    np.testing.assert_allclose(mx.cpu().double().numpy(), Z[np.arange(B), got], rtol=0, atol=2e-5)
    assert not (got == A - 5).any()            # never the later duplicate of 11


@pytest.mark.parametrize("terms,tol", [(3, 1e-4), (1, 8e-3)])
@pytest.mark.parametrize("B,A,HF,nsplit", [(256, 50000, 128, 8), (96, 20011, 64, 16), (64, 5003, 256, 8),
                                           (64, 777, 32, 3)])
def test_screening_argmax_is_exact(B, A, HF, nsplit, terms, tol):
    """rg_flash_amax_screen + rg_flash_argmax_exact (the SQN / SMORL double-Q
    target, sqn_gru.py:222-226): the first maximum of the fp32 logits, also
    where the 3-term (or 1-term, with its wider bound) screening alone would
    pick a different item — planted exact ties (duplicate rows: lowest index)
    and near-ties (1e-6 apart, far below the screening error) — and a row
    with h = 0 (logits = bias)."""
    call, st = C().call, C().stream_ptr()
    g = torch.Generator().manual_seed(A + HF)
    h = torch.tanh(torch.randn(B, HF, generator=g) * 2)
    W = torch.randn(A, HF, generator=g) * 0.3
    b = torch.randn(A, generator=g) * 0.3
    Z = h.double() @ W.double().t() + b.double()
    top = Z.argmax(1)
    for r in range(0, B, 3):        # exact tie: a copy of the winner at a higher index
        j = int(top[r])
        k = (j * 7919 + 13) % A
        if k > j:
            W[k], b[k] = W[j], b[j]
    for r in range(1, B, 3):        # near tie: a slightly better copy at a lower index
        j = int(top[r])
        k = (j * 104729 + 7) % A
        if k < j:
            W[k], b[k] = W[j], b[j] + 1e-6
    h[B - 1] = 0.0                  # every logit of this row = its bias
    b_eq = b.clone()
    hd, Wd, bd = h.to(dev), W.to(dev), b.to(dev)
    rows_eq = B - 1
    Z = h.double() @ W.double().t() + b.double()
    hb, wb = call("rg_head_plane_bytes", B, HF), call("rg_head_plane_bytes", A, HF)
    Hk, Wk = _u8(hb), _u8(wb)
    bp = torch.empty((A + 31) // 32 * 32, device=dev)
    call("rg_head_planes", hd.data_ptr(), B, HF, Hk.data_ptr(), None, None, None, st)
    call("rg_head_planes", Wd.data_ptr(), A, HF, Wk.data_ptr(), None, bd.data_ptr(), bp.data_ptr(), st)
    pbest = torch.empty(nsplit, B, device=dev)
    parg = torch.empty(nsplit, B, dtype=torch.int32, device=dev)
    cmax = torch.empty((A + 31) // 32, B, device=dev)
    call("rg_flash_amax_screen", Hk.data_ptr(), Wk.data_ptr(), bp.data_ptr(), B, A, HF, nsplit, terms,
         pbest.data_ptr(), parg.data_ptr(), cmax.data_ptr(), st)
    idx = torch.empty(B, dtype=torch.int32, device=dev)
    val = torch.empty(B, device=dev)
    call("rg_flash_argmax", pbest.data_ptr(), parg.data_ptr(), nsplit, B, idx.data_ptr(), val.data_ptr(), st)
    wn = torch.empty(1, device=dev)
    call("rg_row_norm_max", Wd.data_ptr(), A, HF, wn.data_ptr(), st)
    cap = call("rg_flash_topk_cap")
    cand = torch.empty(B, cap, dtype=torch.int32, device=dev)
    ncand = torch.empty(B, dtype=torch.int32, device=dev)
    lim = torch.empty(B, device=dev)
    scanned = torch.zeros(1, dtype=torch.int32, device=dev)
    call("rg_flash_argmax_exact", cmax.data_ptr(), B, A, hd.data_ptr(), Wd.data_ptr(), bd.data_ptr(), HF,
         wn.data_ptr(), tol, lim.data_ptr(), cand.data_ptr(), ncand.data_ptr(),
         idx.data_ptr(), val.data_ptr(), scanned.data_ptr(), st)
    torch.cuda.synchronize()
    assert abs(float(wn) - float(W.norm(dim=1).max())) <= 1e-5 * float(W.norm(dim=1).max())
    idx, val = idx.cpu().long(), val.cpu().double()
    # canonical: the first maximum of the fp64 logits (fp32 re-scoring only differs below its own rounding)
    zmax = Z.max(1).values
    first = (Z >= zmax[:, None]).double().argmax(1)
    sl = (h.abs().double() @ W.abs().double().t()).max(1).values   # scale of the row's sums
    for r in range(B):
        if r == rows_eq:
            continue
        if int(idx[r]) != int(first[r]):
            # only within the fp32 re-scoring's own rounding of the two items
            assert float(zmax[r] - Z[r, idx[r]]) <= 200 * 2.0 ** -24 * float(sl[r]), (r, int(idx[r]), int(first[r]))
        assert abs(float(val[r]) - float(Z[r, idx[r]])) <= 200 * 2.0 ** -24 * float(sl[r])
    # exact ties resolve to the lowest index; near ties 1e-6 apart to the better item
    for r in range(0, B - 1, 3):
        assert int(idx[r]) == int(first[r])
    for r in range(1, B - 1, 3):
        assert int(idx[r]) == int(first[r])
    assert int(idx[rows_eq]) == int(torch.argmax(b_eq.double()))


def _tie_flood(B, A, HF, row, step, seed):
    """Inputs where one row's best logits are a flood of exact ties (a copy of
    one W row at every ``step``-th item, far more than the candidate cap)
    plus, at a late copy, a winner larger by ~1e-5 relative that lives in the
    low-order bf16 planes (the 3-product screening does not see it).  The
    other rows are random.  Returns (h, W, b, winner)."""
    g = torch.Generator().manual_seed(seed)
    h = torch.tanh(torch.randn(B, HF, generator=g))
    W = torch.randn(A, HF, generator=g) * 0.3
    b = torch.full((A,), -4.0)
    # aligned with the row's h: the copies' logit (~0.2·Σ|h|) tops every random item's
    copy = 0.3 * torch.sign(h[row]) * (0.5 + 0.5 * torch.rand(HF, generator=g))
    W[::step] = copy
    b[::step] = 0.0
    win = (A - 1) // step * step - step
    W[win] = copy + 2.0 ** -20 * copy.abs() * torch.sign(h[row])
    return h, W, b, win


def test_screening_argmax_overflow_scans_row():
    """A row whose screening band holds more candidate chunks than
    rg_flash_topk_cap() (a flood of exact ties around a winner 1e-5 relative
    above them): the row is scanned whole in fp32 (counted in err) and gets
    the first maximum of its fp32 logits; the other rows are re-scored as
    usual.  (Reference: torch.argmax of the fp32 Q row,
    sqn_gru.py:222-226.)"""
    call, st = C().call, C().stream_ptr()
    B, A, HF, nsplit, row = 64, 5003, 64, 8, 7
    h, W, b, win = _tie_flood(B, A, HF, row, 16, 5)
    hd, Wd, bd = h.to(dev), W.to(dev), b.to(dev)
    hb, wb = call("rg_head_plane_bytes", B, HF), call("rg_head_plane_bytes", A, HF)
    Hk, Wk = _u8(hb), _u8(wb)
    bp = torch.empty((A + 31) // 32 * 32, device=dev)
    call("rg_head_planes", hd.data_ptr(), B, HF, Hk.data_ptr(), None, None, None, st)
    call("rg_head_planes", Wd.data_ptr(), A, HF, Wk.data_ptr(), None, bd.data_ptr(), bp.data_ptr(), st)
    pbest, parg = torch.empty(nsplit, B, device=dev), torch.empty(nsplit, B, dtype=torch.int32, device=dev)
    cmax = torch.empty((A + 31) // 32, B, device=dev)
    call("rg_flash_amax_screen", Hk.data_ptr(), Wk.data_ptr(), bp.data_ptr(), B, A, HF, nsplit, 3, pbest.data_ptr(),
         parg.data_ptr(), cmax.data_ptr(), st)
    idx, val = torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, device=dev)
    call("rg_flash_argmax", pbest.data_ptr(), parg.data_ptr(), nsplit, B, idx.data_ptr(), val.data_ptr(), st)
    wn = torch.empty(1, device=dev)
    call("rg_row_norm_max", Wd.data_ptr(), A, HF, wn.data_ptr(), st)
    cap = call("rg_flash_topk_cap")
    cand, ncand = torch.empty(B, cap, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev)
    lim = torch.empty(B, device=dev)
    scanned = torch.zeros(1, dtype=torch.int32, device=dev)
    call("rg_flash_argmax_exact", cmax.data_ptr(), B, A, hd.data_ptr(), Wd.data_ptr(), bd.data_ptr(), HF,
         wn.data_ptr(), 1e-4, lim.data_ptr(), cand.data_ptr(), ncand.data_ptr(), idx.data_ptr(), val.data_ptr(),
         scanned.data_ptr(), st)
    torch.cuda.synchronize()
    Z = h.double() @ W.double().t() + b.double()
    assert int(ncand[row]) > cap and int(scanned) >= 1
    assert int(idx[row]) == win == int(Z[row].argmax())
    assert torch.equal(idx.cpu().long(), Z.argmax(1))


@pytest.mark.parametrize("K", [1, 5])
def test_fused_topk_overflow_scans_row(K):
    """rg_flash_topk past the candidate cap (the same tie flood in pass 1's
    chunk maxima): the row is scanned whole and its list is the canonical
    (value desc, index asc) top-K of the fp32 logits — the winner, then the
    tied copies in index order; every other row as usual.  Checked bit for bit
    against the canonical order of the native head's fp32 logits of the same
    inputs (rg_head_fwd: the fmaf chain the re-scoring repeats), where the
    planted copies are bitwise equal — so every row, flooded or not, is held
    to the lowest-index tie rule (an fp64 reference splits the copies by its
    BLAS summation order)."""
    call, st = C().call, C().stream_ptr()
    B, A, HF, nsplit, row = 64, 5003, 64, 8, 11
    h, W, b, win = _tie_flood(B, A, HF, row, 16, 9)
    hd, Wd, bd = h.to(dev), W.to(dev), b.to(dev)
    idx, vals, err, _ = run_top(hd, Wd, bd, 6, nsplit, K, exact1=True)
    assert err >= 1
    from recommenders.hip import load_library
    pb = load_library().rg_partial_block()
    nJ, ldz = (A + pb - 1) // pb, (B + 3) // 4 * 4
    ZT = torch.empty(A, ldz, device=dev)
    pm, ps = torch.empty(nJ, B, device=dev), torch.empty(nJ, B, device=dev)
    pa = torch.empty(nJ, B, dtype=torch.int32, device=dev)
    call("rg_head_fwd", hd.data_ptr(), Wd.data_ptr(), bd.data_ptr(), B, A, HF, ZT.data_ptr(), ldz, pm.data_ptr(),
         ps.data_ptr(), pa.data_ptr(), 1, st)
    torch.cuda.synchronize()
    Z32 = ZT[:, :B].t().cpu().numpy()
    # the planted copies are bitwise equal fp32 logits in every row
    assert (Z32[:, 0:A:16][:, :-2] == Z32[:, :1]).all()
    from oracle import metrics as om
    ref = om.canonical_topk(Z32.astype(np.float64), K)
    got = idx.numpy()
    # the flooded row: the winner, then the exactly tied copies in index order
    np.testing.assert_array_equal(got[row], [win] + list(range(0, 16 * (K - 1), 16)))
    # every row: the canonical top-K of the fp32 logits, values bitwise
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(vals.numpy(), np.take_along_axis(Z32, ref, 1).astype(np.float64))


def test_stored_logit_topk_overflow_scans_row():
    """rg_topk over stored logits with more than its 2048 candidates >= tau
    (3000 exact ties at the top of one row): the row is scanned whole, the
    list is the canonical top-K (lowest tied indices), no error raised."""
    call, st = C().call, C().stream_ptr()
    B, A, K = 8, 9001, 20
    g = torch.Generator().manual_seed(2)
    Z = torch.randn(B, A, generator=g)
    Z[3, ::3] = 9.0
    ZT = Z.t().contiguous().to(dev)
    from recommenders.hip import load_library
    pb = load_library().rg_partial_block()
    nJ = (A + pb - 1) // pb
    pmax = torch.stack([Z[:, j * pb:(j + 1) * pb].max(1).values for j in range(nJ)]).contiguous().to(dev)
    idx = torch.empty(B, K, dtype=torch.int32, device=dev)
    vals = torch.empty(B, K, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    call("rg_topk", ZT.data_ptr(), B, pmax.data_ptr(), B, A, K, idx.data_ptr(), vals.data_ptr(), err.data_ptr(), st)
    torch.cuda.synchronize()
    from oracle import metrics as om
    assert int(err) == 0
    np.testing.assert_array_equal(idx.cpu().numpy(), om.canonical_topk(Z.numpy(), K))
    assert (idx[3].cpu() == torch.arange(0, 3 * K, 3, dtype=torch.int32)).all()


def test_screening_argmax_row_chunks_match(monkeypatch):
    """SoftmaxHead.argmax on the split path: screening in row chunks (what C5
    at one GPU does when the chunk maxima would exceed SCREEN_CMAX_BYTES)
    gives the same items and values as one whole-batch screening, and both
    equal the fp64 first maximum away from fp32 rounding ties."""
    from recommenders.hip import engine
    B, A, HF = 1024, 20000, 128
    hd = engine.SoftmaxHead("x", A, HF, dev)
    hd.set_matmul_precision("f32x6")
    g = torch.Generator().manual_seed(3)
    h = torch.tanh(torch.randn(B, HF, generator=g)).to(dev)
    i1 = hd.argmax(h, slot="a").clone()
    v1 = hd.argmax_mx.clone()
    monkeypatch.setattr(engine, "SCREEN_CMAX_BYTES", 1)
    monkeypatch.setattr(engine, "SCREEN_ROW_CHUNK", 256)
    i2 = hd.argmax(h, slot="b").clone()
    v2 = hd.argmax_mx.clone()
    assert hd._aws["b"].Bc == 256
    assert torch.equal(i1, i2) and torch.equal(v1, v2)
    Z = h.double().cpu() @ hd.W.p.double().cpu().t() + hd.b.p.double().cpu()
    zmax = Z.max(1).values
    gap = zmax - Z[torch.arange(B), i1.cpu().long()]
    assert float(gap.max()) <= 1e-5


def _plant_top1_ties(h, W, b, Z):
    """Exact ties (a copy of a row's winner at a higher index) and near ties
    (a copy 1e-6 better at a lower index) for every third row."""
    A = W.shape[0]
    top = Z.argmax(1)
    for r in range(0, h.shape[0], 3):
        j = int(top[r])
        k = (j * 7919 + 13) % A
        if k > j:
            W[k], b[k] = W[j], b[j]
    for r in range(1, h.shape[0], 3):
        j = int(top[r])
        k = (j * 104729 + 7) % A
        if k < j:
            W[k], b[k] = W[j], b[j] + 1e-6


def _head_top1(A, HF, h, W, b):
    from recommenders.hip import engine
    hd = engine.SoftmaxHead("sup", A, HF, dev)
    hd.set_matmul_precision("f32x6d3")
    with torch.no_grad():
        hd.W.p.copy_(W)
        hd.b.p.copy_(b)
    hd.top_k = 1
    tgt = torch.zeros(h.shape[0], dtype=torch.int64, device=dev)
    _, w = hd.forward_loss(h, tgt, slot="main")
    idx, val = hd.top_entries(w)
    torch.cuda.synchronize()
    return hd, w, idx[:, 0].clone(), val[:, 0].clone()


def test_top1_row_chunked_screening_matches_chunk_maxima(monkeypatch):
    """SMORL's K = 1 reward item when pass 1's chunk maxima would exceed
    SCREEN_CMAX_BYTES (C5 on one GPU): the row-chunked screening argmax on
    pass 1's planes + fp32 re-scoring gives the same items and values as the
    chunk-maxima path (both the first maximum of the fp32 logits)."""
    from recommenders.hip import engine
    B, A, HF = 1024, 20011, 128
    g = torch.Generator().manual_seed(17)
    h = torch.tanh(torch.randn(B, HF, generator=g))
    W, b = torch.randn(A, HF, generator=g) * 0.3, torch.randn(A, generator=g) * 0.3
    _plant_top1_ties(h, W, b, h.double() @ W.double().t() + b.double())
    hd1, w1, i1, v1 = _head_top1(A, HF, h.to(dev), W.to(dev), b.to(dev))
    assert w1.top1 is None   # the chunk-maxima path (its view is dropped after top_entries)
    # no room for the (shared) chunk maxima: the screening fallback, in 256-row chunks
    monkeypatch.setattr(engine, "CMAX_FREE_MARGIN", 1 << 62)
    monkeypatch.setattr(engine, "_CMAX", {})
    monkeypatch.setattr(engine, "SCREEN_CMAX_BYTES", 1)
    monkeypatch.setattr(engine, "SCREEN_ROW_CHUNK", 256)
    hd2, w2, i2, v2 = _head_top1(A, HF, h.to(dev), W.to(dev), b.to(dev))
    assert w2.cmax is None and w2.top1 is not None and w2.top1.Bc == 256
    assert torch.equal(i1, i2) and torch.equal(v1, v2)
    Z = h.double() @ W.double().t() + b.double()
    first = (Z >= Z.max(1).values[:, None]).double().argmax(1)
    for r in range(0, B, 3):
        assert int(i2[r]) == int(first[r])
    for r in range(1, B, 3):
        assert int(i2[r]) == int(first[r])


def test_top1_above_2gb_of_chunk_maxima_is_first_fp32_maximum(monkeypatch):
    """The K = 1 screening fallback (no room for pass 1's chunk maxima) at a
    size whose chunk maxima really exceed 2 GB (A = 2M, B = 8704: 2.18 GB,
    screened in 2048-row chunks): planted exact / 1e-6 near ties resolve to
    the first maximum of the fp32 logits (fp64 first maximum, away from fp32
    rounding of the two items)."""
    from recommenders.hip import engine
    monkeypatch.setattr(engine, "CMAX_FREE_MARGIN", 1 << 62)
    monkeypatch.setattr(engine, "_CMAX", {})
    B, A, HF = 8704, 2_000_000, 32
    assert -(-A // 32) * B * 4 > 2 << 30
    g = torch.Generator(device=dev).manual_seed(23)
    h = torch.tanh(torch.randn(B, HF, generator=g, device=dev))
    W = torch.randn(A, HF, generator=g, device=dev) * 0.3
    b = torch.randn(A, generator=g, device=dev) * 0.3
    top = torch.cat([(h[r0:r0 + 512].double() @ W.double().t() + b.double()).argmax(1)
                     for r0 in range(0, B, 512)]).cpu()
    Wc, bc = W.cpu(), b.cpu()
    for r in range(0, 600, 3):
        j = int(top[r])
        k = (j * 7919 + 13) % A
        if k > j:
            Wc[k], bc[k] = Wc[j], bc[j]
    for r in range(1, 600, 3):
        j = int(top[r])
        k = (j * 104729 + 7) % A
        if k < j:
            Wc[k], bc[k] = Wc[j], bc[j] + 1e-6
    W, b = Wc.to(dev), bc.to(dev)
    hd, w, idx, val = _head_top1(A, HF, h, W, b)
    assert w.cmax is None and w.top1 is not None
    del w
    hd.release_eval()
    for r0 in range(0, B, 512):
        Z = h[r0:r0 + 512].double() @ W.double().t() + b.double()
        zmax = Z.max(1).values
        first = (Z >= zmax[:, None]).double().argmax(1)
        got = idx[r0:r0 + 512].long()
        gap = zmax - Z.gather(1, got[:, None])[:, 0]
        sl = (h[r0:r0 + 512].abs().double() @ W.abs().double().t()).max(1).values
        bad = (got != first) & (gap > 200 * 2.0 ** -24 * sl)
        assert not bool(bad.any()), r0
        if r0 == 0:   # the planted rows: exactly the first maximum
            assert torch.equal(got[:600], first[:600])
        torch.testing.assert_close(val[r0:r0 + 512].double(), Z.gather(1, got[:, None])[:, 0],
                                   rtol=0, atol=float(200 * 2.0 ** -24 * sl.max()))


@pytest.mark.parametrize("B,A,HF,zs", [(128, 3001, 64, False), (256, 20011, 128, True), (128, 5003, 256, True)])
def test_chunk_maxima_without_first_maximum_match(B, A, HF, zs):
    """rg_flash_fwd_top with cmax alone (the trainers' fused top-k: no per-logit
    compare-and-select of the first maximum) writes the same chunk maxima,
    softmax partials, O partials and stored logits, bit for bit, as with
    pbest / parg too."""
    call, st = C().call, C().stream_ptr()
    h, W, b, _ = inputs(B, A, HF, 11 * B + A)
    h, W, b = h.to(dev), W.to(dev), b.to(dev)
    nsplit = 8
    hb, wb = call("rg_head_plane_bytes", B, HF), call("rg_head_plane_bytes", A, HF)
    Hk, Hr, Wk, Wr = _u8(hb), _u8(hb), _u8(wb), _u8(wb)
    bp = torch.empty((A + 31) // 32 * 32, device=dev)
    call("rg_head_planes", h.data_ptr(), B, HF, Hk.data_ptr(), Hr.data_ptr(), None, None, st)
    call("rg_head_planes", W.data_ptr(), A, HF, Wk.data_ptr(), Wr.data_ptr(), b.data_ptr(), bp.data_ptr(), st)
    outs = []
    for full in (True, False):
        z = lambda *s, dt=torch.float32: torch.full(s, -7, dtype=dt, device=dev)  # noqa: E731
        pm, pl, pO, cmax = z(nsplit, B), z(nsplit, B), z(nsplit, HF, B), z((A + 31) // 32, B)
        pbest, parg = (z(nsplit, B), z(nsplit, B, dt=torch.int32)) if full else (None, None)
        zbuf = torch.zeros(call("rg_flash_zs_bytes", B, A) // 4, device=dev) if zs else None
        call("rg_flash_fwd_top", Hk.data_ptr(), Wk.data_ptr(), Wr.data_ptr(), bp.data_ptr(), B, A, HF, 636, nsplit,
             pm.data_ptr(), pl.data_ptr(), pO.data_ptr(), None if pbest is None else pbest.data_ptr(),
             None if parg is None else parg.data_ptr(), cmax.data_ptr(), None if zbuf is None else zbuf.data_ptr(), st)
        outs.append([pm, pl, pO, cmax] + ([zbuf] if zs else []))
    torch.cuda.synchronize()
    for a_, b_ in zip(*outs):
        assert torch.equal(a_, b_)
