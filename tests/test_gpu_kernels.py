"""Per-kernel GPU numerics through the C ABI, each against a plain PyTorch
(CPU, fp64 where it matters) reference of the same op."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"


def C():
    from recommenders import hip
    return hip


def st():
    return C().stream_ptr()


_KEEP = []


def D(t):
    """Device copy kept alive for the whole test (a temporary's block would be
    recycled by the caching allocator before an async kernel reads it)."""
    d = t.to(dev)
    _KEEP.append(d)
    return d


def pack(lens, L, unpacked=0):
    B = lens.numel()
    perm = torch.empty(B, dtype=torch.int32, device=dev)
    ls = torch.empty(B, dtype=torch.int32, device=dev)
    offs = torch.empty(B + 1, dtype=torch.int32, device=dev)
    C().call("rg_pack", D(lens).data_ptr(), B, L, unpacked, perm.data_ptr(), ls.data_ptr(), offs.data_ptr(),
             st())
    return perm, ls, offs


def test_pack_stable_descending():
    g = torch.Generator().manual_seed(0)
    # B <= 8192: the bitonic-sort kernel; 9000: the general one; lengths outside [1, L] clamp
    for B, L in [(7, 5), (1000, 20), (4096, 50), (3000, 3), (8192, 100), (9000, 30), (1, 4), (4096, 512)]:
        lens = torch.randint(1, L + 1, (B,), generator=g)
        if B > 1:
            lens[0], lens[-1] = 0, L + 7
        perm, ls, offs = pack(lens, L)
        lc = lens.clamp(1, L).numpy()
        order = np.argsort(-lc, kind="stable")
        assert np.array_equal(perm.cpu().numpy(), order)
        assert np.array_equal(ls.cpu().numpy(), lc[order])
        assert np.array_equal(offs.cpu().numpy(), np.concatenate([[0], np.cumsum(lc[order])]))
        perm, ls, offs = pack(lens, L, unpacked=1)
        assert int(offs[-1]) == B * L


@pytest.mark.parametrize("B,L,N,E", [(33, 6, 100, 16),
                                     # k_gather_e's long / short sorted-row pairing (B % 4 == 0) and the
                                     # general form (B % 4 != 0) at every table width it takes
                                     (256, 50, 5000, 32), (252, 50, 5000, 64), (512, 50, 20000, 128),
                                     (130, 40, 3000, 128), (96, 20, 2000, 256), (101, 20, 2000, 256)])
def test_gather_packed_and_reverse(B, L, N, E):
    g = torch.Generator().manual_seed(1 + B + E)
    s = torch.randint(0, N + 1, (B, L), generator=g)
    lens = torch.randint(1, L + 1, (B,), generator=g)
    emb = torch.randn(N + 1, E, generator=g)
    perm, ls, offs = pack(lens, L)
    for rev in (0, 1):
        X = torch.zeros(B * L, E, device=dev)
        ids = torch.zeros(B * L, dtype=torch.int32, device=dev)
        C().call("rg_gather", D(s).data_ptr(), B, L, perm.data_ptr(), ls.data_ptr(), offs.data_ptr(),
                 D(emb).data_ptr(), N + 1, E, rev, ids.data_ptr(), X.data_ptr(), None, st())
        rows = []
        for r in perm.cpu().tolist():
            t = list(range(int(lens[r])))
            if rev:
                t = t[::-1]
            rows += [int(s[r, i]) for i in t]
        T = len(rows)
        assert ids[:T].cpu().tolist() == rows
        torch.testing.assert_close(X[:T].cpu(), emb[rows], rtol=0, atol=0)


@pytest.mark.parametrize("M,N,K,splits", [(100, 384, 128, 1), (1000, 96, 32, 1), (384, 128, 5000, 8),
                                          (48, 16, 37, 3)])
def test_gemm_layouts(M, N, K, splits):
    g = torch.Generator().manual_seed(2)
    A = torch.randn(M, K, generator=g)
    Bm = torch.randn(K, N, generator=g)
    ref = (A.double() @ Bm.double()).float()
    Ad, Bd = A.to(dev), Bm.to(dev)
    AT, BT = A.t().contiguous().to(dev), Bm.t().contiguous().to(dev)
    for (a, sam, sak) in ((Ad, K, 1), (AT, 1, M)):
        for (b, sbk, sbn) in ((Bd, N, 1), (BT, 1, K)):
            out = torch.zeros(splits, M, N, device=dev)
            C().call("rg_gemm_f32", a.data_ptr(), sam, sak, b.data_ptr(), sbk, sbn, out.data_ptr(), N, None, M,
                     None, N, K, None, splits, st())
            torch.testing.assert_close(out.sum(0).cpu(), ref, rtol=1e-5, atol=1e-4 * max(1.0, K / 1000))


@pytest.mark.parametrize("M,N,K", [(85003, 384, 128), (300, 128, 384), (129, 768, 256), (7, 256, 32), (4100, 60, 64)])
def test_gemm_large_tile_path(M, N, K):
    """k_gemm_nt (rg_gemm_f32 with A k-contiguous, no split-K, K % 32 == 0):
    both B layouts, bias, the row count read from the device (grid sized
    for more rows than exist), partial M / N tiles, against fp64."""
    g = torch.Generator().manual_seed(4)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) * 0.1
    bias = torch.randn(N, generator=g)
    ref = (A.double() @ W.double().t() + bias.double()).float()
    Ad, bd = A.to(dev), bias.to(dev)
    Mdev = torch.tensor([M], dtype=torch.int32, device=dev)
    for Bd, sbk, sbn in ((W.to(dev), 1, K), (W.t().contiguous().to(dev), N, 1)):
        out = torch.full((M + 5, N), float("nan"), device=dev)
        C().call("rg_gemm_f32", Ad.data_ptr(), K, 1, Bd.data_ptr(), sbk, sbn, out.data_ptr(), N, bd.data_ptr(),
                 M + 200, Mdev.data_ptr(), N, K, None, 1, st())
        torch.testing.assert_close(out[:M].cpu(), ref, rtol=1e-5, atol=1e-4 * max(1.0, K / 1000))
        assert torch.isnan(out[M:]).all()   # rows past the device-side count untouched


def gru_ref(X_rows, lens, perm_order, Wih, Whh, bih, bhh, H):
    """fp64 GRU over each (unsorted) row; returns final h per original row and saved states."""
    hs = {}
    for r, xs in X_rows.items():
        h = torch.zeros(H, dtype=torch.float64)
        for x in xs:
            gi = Wih @ x + bih
            gh = Whh @ h + bhh
            rr = torch.sigmoid(gi[:H] + gh[:H])
            zz = torch.sigmoid(gi[H:2 * H] + gh[H:2 * H])
            nn_ = torch.tanh(gi[2 * H:] + rr * gh[2 * H:])
            h = (1 - zz) * nn_ + zz * h
        hs[r] = h
    return hs


@pytest.mark.parametrize("H,B,L", [(16, 37, 7), (32, 37, 7), (64, 37, 7), (128, 37, 7), (256, 37, 7),
                                   (256, 77, 23)])
def test_gru_forward_backward(H, B, L):
    """H = 256: the persistent wide path (W_hh streamed from L2 as MFMA
    fragments, 32 rows per workgroup; partial last workgroup at B = 37, 77)."""
    wide = H == 256
    g = torch.Generator().manual_seed(3 + L)
    E = H
    lens = torch.randint(1, L + 1, (B,), generator=g)
    X = torch.randn(B, L, E, generator=g) * 0.5
    k = 1 / H ** 0.5
    Wih = (torch.rand(3 * H, E, generator=g) * 2 - 1) * k
    Whh = (torch.rand(3 * H, H, generator=g) * 2 - 1) * k
    bih = (torch.rand(3 * H, generator=g) * 2 - 1) * k
    bhh = (torch.rand(3 * H, generator=g) * 2 - 1) * k
    perm, ls, offs = pack(lens, L)
    order = perm.cpu().tolist()
    packed = torch.cat([X[r, :int(lens[r])] for r in order])
    T = packed.shape[0]
    Gi = (packed.double() @ Wih.double().t() + bih.double()).float().to(dev)
    hout = torch.zeros(B, H, device=dev)
    saved = torch.zeros(5, T, H, device=dev)
    work = torch.zeros(C().call("rg_gru_wide_work_bytes", H) // 4 if wide else 1, device=dev)
    if wide:
        C().call("rg_gru_fwd_wide", Gi.data_ptr(), D(Whh).data_ptr(), D(bhh).data_ptr(), perm.data_ptr(),
                 ls.data_ptr(), offs.data_ptr(), B, H, hout.data_ptr(), H, 0, saved.data_ptr(), T * H,
                 work.data_ptr(), st())
    else:
        C().call("rg_gru_fwd", Gi.data_ptr(), D(Whh).data_ptr(), D(bhh).data_ptr(), perm.data_ptr(),
                 ls.data_ptr(), offs.data_ptr(), B, H, hout.data_ptr(), H, 0, saved.data_ptr(), T * H, st())
    # autograd reference (float64)
    Xd = X.double().requires_grad_(True)
    P = [t.double().requires_grad_(True) for t in (Wih, Whh, bih, bhh)]
    hs = []
    for r in range(B):
        h = torch.zeros(H, dtype=torch.float64)
        for t in range(int(lens[r])):
            gi = P[0] @ Xd[r, t] + P[2]
            gh = P[1] @ h + P[3]
            rr = torch.sigmoid(gi[:H] + gh[:H])
            zz = torch.sigmoid(gi[H:2 * H] + gh[H:2 * H])
            nn_ = torch.tanh(gi[2 * H:] + rr * gh[2 * H:])
            h = (h - nn_) * zz + nn_
        hs.append(h)
    href = torch.stack(hs)
    torch.testing.assert_close(hout.cpu().double(), href.detach(), rtol=0, atol=2e-6)
    dh = torch.randn(B, H, generator=g)
    (href * dh.double()).sum().backward()
    dGi = torch.zeros(T, 3 * H, device=dev)
    dGh = torch.zeros(T, 3 * H, device=dev)
    if wide:
        C().call("rg_gru_bwd_wide", saved.data_ptr(), T * H, D(Whh).data_ptr(), perm.data_ptr(), ls.data_ptr(),
                 offs.data_ptr(), B, H, D(dh).data_ptr(), H, 0, dGi.data_ptr(), dGh.data_ptr(), work.data_ptr(),
                 st())
    else:
        C().call("rg_gru_bwd", saved.data_ptr(), T * H, D(Whh).data_ptr(), perm.data_ptr(), ls.data_ptr(),
                 offs.data_ptr(), B, H, D(dh).data_ptr(), H, 0, dGi.data_ptr(), dGh.data_ptr(), st())
    # dX = dGi · W_ih (packed order) vs autograd
    dX = (dGi.cpu().double() @ Wih.double())
    ref_dX = torch.cat([Xd.grad[r, :int(lens[r])] for r in order])
    torch.testing.assert_close(dX, ref_dX, rtol=0, atol=2e-5)
    dWhh = dGh.cpu().double().t() @ saved[0].cpu().double()
    torch.testing.assert_close(dWhh, P[1].grad, rtol=0, atol=5e-5)
    torch.testing.assert_close(dGh.cpu().double().sum(0), P[3].grad, rtol=0, atol=5e-5)
    torch.testing.assert_close(dGi.cpu().double().sum(0), P[2].grad, rtol=0, atol=5e-5)


@pytest.mark.parametrize("B,A,HF", [(64, 1000, 16), (100, 3000, 32), (256, 5000, 64), (260, 20000, 128),
                                    (96, 4100, 256)])
def test_head_forward_backward(B, A, HF):
    g = torch.Generator().manual_seed(4)
    h = torch.randn(B, HF, generator=g) * 0.5
    W = torch.randn(A, HF, generator=g) * 0.1
    b = torch.randn(A, generator=g) * 0.1
    tgt = torch.randint(0, A, (B,), generator=g)
    hd, Wd, bd, td = h.to(dev), W.to(dev), b.to(dev), tgt.to(dev)
    ldz = (B + 3) // 4 * 4
    pb = C().load_library().rg_partial_block()
    nJ = (A + pb - 1) // pb
    ZT = torch.zeros(A, ldz, device=dev)
    pm = torch.zeros(nJ, B, device=dev)
    ps = torch.zeros(nJ, B, device=dev)
    pa = torch.zeros(nJ, B, dtype=torch.int32, device=dev)
    C().call("rg_head_fwd", hd.data_ptr(), Wd.data_ptr(), bd.data_ptr(), B, A, HF, ZT.data_ptr(), ldz,
             pm.data_ptr(), ps.data_ptr(), pa.data_ptr(), 1, st())
    Zref = (h.double() @ W.double().t() + b.double())
    torch.testing.assert_close(ZT[:, :B].t().cpu().double(), Zref, rtol=0, atol=1e-5)
    work = torch.zeros(3 * min(128, nJ) * B, device=dev)
    lse = torch.zeros(B, device=dev)
    amax = torch.zeros(B, dtype=torch.int32, device=dev)
    lrow = torch.zeros(B, device=dev)
    mx = torch.zeros(B, device=dev)
    C().call("rg_lse_combine", pm.data_ptr(), ps.data_ptr(), pa.data_ptr(), B, nJ, work.data_ptr(), ZT.data_ptr(),
             ldz, td.data_ptr(), A, lse.data_ptr(), amax.data_ptr(), lrow.data_ptr(), mx.data_ptr(), st())
    torch.testing.assert_close(lse.cpu().double(), torch.logsumexp(Zref, 1), rtol=0, atol=2e-5)
    # the row maximum is the exact stored logit at the argmax
    np.testing.assert_array_equal(mx.cpu().numpy(), ZT[:, :B].t().cpu().max(1).values.numpy())
    Zg = ZT[:, :B].t().cpu()
    assert torch.equal(amax.cpu().long(), torch.argmax(Zg, 1))
    ce = torch.nn.functional.cross_entropy(Zref, tgt, reduction="none")
    torch.testing.assert_close(lrow.cpu().double(), ce, rtol=0, atol=2e-5)
    # backward w.r.t. h, W, b (grad-only hook of the fused Adam kernel)
    Wr = W.double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    hr = h.double().requires_grad_(True)
    torch.nn.functional.cross_entropy(hr @ Wr.t() + br, tgt).backward()
    gs = float(np.float32(1.0 / B))
    splits = 8
    slabs = torch.zeros(splits, B, HF, device=dev)
    n = C().call("rg_head_dh", ZT.data_ptr(), ldz, lse.data_ptr(), td.data_ptr(), gs, Wd.data_ptr(), B, A, HF,
                 splits, slabs.data_ptr(), st())
    torch.testing.assert_close(slabs[:n].sum(0).cpu().double(), hr.grad, rtol=0, atol=1e-6)
    dW = torch.zeros(A, HF, device=dev)
    db = torch.zeros(A, device=dev)
    C().call("rg_head_dw_adam", ZT.data_ptr(), ldz, lse.data_ptr(), td.data_ptr(), gs, hd.data_ptr(), B, A, HF,
             None, None, None, None, None, None, None, dW.data_ptr(), db.data_ptr(), st())
    torch.testing.assert_close(dW.cpu().double(), Wr.grad, rtol=0, atol=1e-7)
    torch.testing.assert_close(db.cpu().double(), br.grad, rtol=0, atol=1e-7)


@pytest.mark.parametrize("rows,cols,offset", [(300, 16, 0), (303, 1, 0), (300, 1, 0), (3, 1, 0), (301, 3, 0),
                                             (300, 1, 1), (300, 16, 1)])
def test_adam_kernels_match_torch(rows, cols, offset):
    """Row-sparse Adam: wide rows (f4), one-column tables (the heads' biases:
    four rows per thread plus the tail; offset 1: tensors not 16-B aligned take
    the scalar path), other widths (scalar)."""
    from recommenders.hip.engine import AdamClock
    g = torch.Generator().manual_seed(5)
    p0 = torch.randn(rows, cols, generator=g)
    grads = [torch.randn(rows, cols, generator=g) for _ in range(3)]
    touched = [torch.rand(rows, generator=g) < 0.3 for _ in range(3)]
    pt = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([pt], lr=0.01)
    P = torch.empty(rows * cols + offset, device=dev)[offset:].view(rows, cols)
    P.copy_(p0)
    M = torch.zeros(rows * cols + offset, device=dev)[offset:].view(rows, cols)
    V = torch.zeros(rows * cols + offset, device=dev)[offset:].view(rows, cols)
    G = torch.zeros(rows * cols + offset, device=dev)[offset:].view(rows, cols)
    tags = torch.zeros(rows + offset, dtype=torch.int32, device=dev)[offset:]
    clock = AdamClock(0.01)
    for i in range(3):
        gi = grads[i] * touched[i].float().unsqueeze(1)
        pt.grad = gi.clone()
        opt.step()
        G[touched[i].to(dev)] = gi[touched[i]].to(dev)
        tags[touched[i].to(dev)] = i + 1
        C().call("rg_adam_rows", P.data_ptr(), M.data_ptr(), V.data_ptr(), G.data_ptr(), tags.data_ptr(), i + 1,
                 rows, cols, clock.next_args(), st())
    torch.testing.assert_close(P.cpu(), pt.detach(), rtol=0, atol=2e-6)
    assert float(G.abs().max()) == 0.0


@pytest.mark.parametrize("n,nslab", [(49152, 128), (384, 128), (1000, 7), (33, 1)])
def test_adam_slabs_match_torch(n, nslab):
    """Split-K slab reduction + Adam (the GRU weights' update): gradient = Σ
    slabs (fp64 reference), the step as torch.optim.Adam; g_out mode returns
    the reduced gradient; two launches are bitwise identical."""
    from recommenders.hip.engine import AdamClock
    g = torch.Generator().manual_seed(9)
    p0 = torch.randn(n, generator=g)
    slabs = [torch.randn(nslab, n, generator=g) * 0.1 for _ in range(2)]
    pt = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([pt], lr=0.01)
    P, M, V = p0.to(dev), torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    clock = AdamClock(0.01)
    for i in range(2):
        pt.grad = slabs[i].double().sum(0).float()
        opt.step()
        C().call("rg_adam_slabs", P.data_ptr(), M.data_ptr(), V.data_ptr(), D(slabs[i]).data_ptr(), nslab, n,
                 clock.next_args(), None, st())
    torch.testing.assert_close(P.cpu(), pt.detach(), rtol=0, atol=2e-6)
    out = [torch.empty(n, device=dev) for _ in range(2)]
    sd = D(slabs[0])
    for o in out:
        C().call("rg_adam_slabs", P.data_ptr(), M.data_ptr(), V.data_ptr(), sd.data_ptr(), nslab, n, None,
                 o.data_ptr(), st())
    torch.testing.assert_close(out[0].cpu().double(), slabs[0].double().sum(0), rtol=0, atol=1e-5)
    assert torch.equal(out[0], out[1])


def test_q_kernels_and_rewards():
    g = torch.Generator().manual_seed(6)
    B, A, HF, Ed = 50, 400, 32, 8
    h = torch.randn(B, HF, generator=g)
    Ws = [torch.randn(A, HF, generator=g) for _ in range(3)]
    bs = [torch.randn(A, generator=g) for _ in range(3)]
    idx = torch.randint(0, A, (B,), generator=g)
    hd = h.to(dev)
    Wd = [w.to(dev) for w in Ws]
    bd = [b.to(dev) for b in bs]
    q = torch.zeros(B, 3, device=dev)
    hip = C()
    hip.call("rg_q_gather", hd.data_ptr(), HF, hip.host_ptr_array(Wd), hip.host_ptr_array(bd), 3,
             D(idx).data_ptr(), None, B, q.data_ptr(), st())
    ref = torch.stack([(h * Ws[i][idx]).sum(1) + bs[i][idx] for i in range(3)], 1)
    torch.testing.assert_close(q.cpu(), ref, rtol=0, atol=1e-5)
    # backward: dh += Σ_i dq_i W_i[a]; G_i[a] += dq_i h, Gb_i[a] += dq_i through the sorted scatter
    # (many rows share an action: idx drawn from 7 actions), -1 rows skipped; bitwise repeatable
    from recommenders.hip.qlearn import q_heads_backward

    class _QH:
        def __init__(self, W):
            self.W = type("P", (), {"p": W})()
            self.A = A
            self.G = torch.zeros(A, HF, device=dev)
            self.Gb = torch.zeros(A, device=dev)
            self.tags = torch.zeros(A, dtype=torch.int32, device=dev)

    class _Main:
        def __init__(self):
            self.q_heads = [_QH(w) for w in Wd]
            self.hf, self.device, self._b = HF, dev, {}

        def buf(self, name, shape, dtype=torch.float32):
            t = self._b.get(name)
            if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
                t = self._b[name] = torch.empty(*shape, dtype=dtype, device=dev)
            return t

    ib = torch.randint(0, 7, (B,), generator=g) * 37
    ib[3] = -1
    dq = torch.randn(B, 3, generator=g)
    dh0 = torch.randn(B, HF, generator=g)
    outs = []
    for rep in range(2):
        mn = _Main()
        dh = dh0.to(dev)
        q_heads_backward(mn, hd, D(ib), B, D(dq), dh, 5, st())
        torch.cuda.synchronize()
        outs.append((dh.cpu(), [x.G.cpu() for x in mn.q_heads], [x.Gb.cpu() for x in mn.q_heads],
                     [x.tags.cpu() for x in mn.q_heads]))
    ok = ib >= 0
    dh_ref = dh0.double().clone()
    for i in range(3):
        dh_ref[ok] += dq[ok, i:i + 1].double() * Ws[i][ib[ok]].double()
        Gr = torch.zeros(A, HF, dtype=torch.float64).index_add_(0, ib[ok], dq[ok, i:i + 1].double() * h[ok].double())
        Gbr = torch.zeros(A, dtype=torch.float64).index_add_(0, ib[ok], dq[ok, i].double())
        torch.testing.assert_close(outs[0][1][i].double(), Gr, rtol=0, atol=1e-5)
        torch.testing.assert_close(outs[0][2][i].double(), Gbr, rtol=0, atol=1e-5)
        tg = torch.zeros(A, dtype=torch.int32)
        tg[ib[ok]] = 5
        assert torch.equal(outs[0][3][i], tg)
        assert torch.equal(outs[0][1][i], outs[1][1][i]) and torch.equal(outs[0][2][i], outs[1][2][i])
    torch.testing.assert_close(outs[0][0].double(), dh_ref, rtol=0, atol=1e-5)
    assert torch.equal(outs[0][0], outs[1][0])
    # diversity / novelty
    from oracle import metrics as om
    L = 5
    s = torch.randint(0, A, (B, L), generator=g)
    lens = torch.randint(1, L + 1, (B,), generator=g)
    table = torch.randn(A + 1, Ed, generator=g)
    preds = torch.randn(B, A, generator=g)
    top = torch.topk(preds, 3).indices.to(torch.int32)
    out = torch.zeros(B, device=dev)
    hip.call("rg_diversity", D(s).data_ptr(), L, D(lens).data_ptr(), 1, D(top).data_ptr(), 3, 3,
             D(table).data_ptr(), table.shape[0], Ed, 1e-6, B, out.data_ptr(), st())
    torch.testing.assert_close(out.cpu(), om.batch_diversity_rewards(s, preds, lens, "end", 3, table), rtol=0,
                               atol=1e-6)
    unpop = set(range(0, A, 3))
    bm = np.zeros((A + 31) // 32, dtype=np.uint32)
    for j in unpop:
        bm[j >> 5] |= np.uint32(1 << (j & 31))
    outn = torch.zeros(B, device=dev)
    bmd = D(torch.from_numpy(bm.view(np.int32)))
    hip.call("rg_novelty", D(top).data_ptr(), 3, 3, bmd.data_ptr(), A, 2.0, B, outn.data_ptr(), st())
    np.testing.assert_allclose(outn.cpu().numpy(), om.batch_novelty_rewards(preds, unpop, 2.0, 3), atol=1e-6)
    # an id outside [0, A) (never a real prediction): NaN for that row, no bitmap read
    bad = top.clone()
    bad[0, 1], bad[1, 0] = -1, A + 40
    hip.call("rg_novelty", D(bad).data_ptr(), 3, 3, bmd.data_ptr(), A, 2.0, B, outn.data_ptr(), st())
    o = outn.cpu().numpy()
    assert np.isnan(o[:2]).all() and not np.isnan(o[2:]).any()


@pytest.mark.parametrize("M,N,T,splits", [(384, 128, 5000, 16), (48, 16, 77, 3), (192, 64, 3000, 128)])
def test_wgrad_fused_bias(M, N, T, splits):
    g = torch.Generator().manual_seed(7)
    G = torch.randn(T + 40, M, generator=g)
    X = torch.randn(T + 40, N, generator=g)
    Tdev = D(torch.tensor([T], dtype=torch.int32))
    dw = torch.zeros(splits, M, N, device=dev)
    db = torch.zeros(splits, M, device=dev)
    C().call("rg_wgrad", D(G).data_ptr(), M, D(X).data_ptr(), N, T + 40, Tdev.data_ptr(), splits, dw.data_ptr(),
             db.data_ptr(), st())
    ref = G[:T].double().t() @ X[:T].double()
    torch.testing.assert_close(dw.sum(0).cpu().double(), ref, rtol=0, atol=2e-6 * T)
    torch.testing.assert_close(db.sum(0).cpu().double(), G[:T].double().sum(0), rtol=0, atol=2e-6 * T)


@pytest.mark.parametrize("E,n_rows,n,n_max", [(128, 1000, 20000, 24000), (32, 50, 3000, 3000), (256, 7000, 5000, 6400),
                                              (1, 300, 777, 1000)])
def test_scatter_rows_deterministic(E, n_rows, n, n_max):
    """rg_scatter_rows (csrc/segsum.hip): G[id] += src rows for the first n of
    n_max rows, skipping skip_id / invalid ids — one heavy id whose run spans
    many 64-position blocks, runs ending exactly on block edges, -1 and
    out-of-range ids; equals an fp64 index_add within fp32 rounding, tags the
    touched rows, and two runs are bitwise identical."""
    g = torch.Generator().manual_seed(E + n)
    ids = torch.randint(0, n_rows, (n_max,), generator=g, dtype=torch.int32)
    ids[: n // 4] = 7                                   # heavy hitter: a long run across blocks
    ids[n // 4: n // 4 + 64] = 3                        # a run of exactly one block
    ids[5] = -1
    ids[6] = n_rows + 5
    skip = 11 % n_rows
    ids[n // 2: n // 2 + 10] = skip
    ids = ids[torch.randperm(n_max, generator=g)]
    src = torch.randn(n_max, E, generator=g)
    n_t = torch.tensor([n], dtype=torch.int32, device=dev)
    nb = C().call("rg_scatter_rows_work_bytes", n_max, E, n_rows)
    work = torch.empty(nb, dtype=torch.uint8, device=dev)
    outs = []
    for rep in range(2):
        G = torch.zeros(n_rows, E, device=dev)
        G[0] = 1.0                                      # adds, not overwrites
        tags = torch.zeros(n_rows, dtype=torch.int32, device=dev)
        C().call("rg_scatter_rows", D(ids).data_ptr(), D(src).data_ptr(), E, E, n_t.data_ptr(), n_max, skip,
                 G.data_ptr(), n_rows, tags.data_ptr(), 9, 0, work.data_ptr(), nb, st())
        # a second source over the same rows reuses the sort (the sampled head's bias): column 0 of
        # the same rows, read with the row stride E
        G1 = torch.zeros(n_rows, 1, device=dev)
        C().call("rg_scatter_rows", D(ids).data_ptr(), D(src).data_ptr(), 1, E, n_t.data_ptr(),
                 n_max, skip, G1.data_ptr(), n_rows, tags.data_ptr(), 9, 1, work.data_ptr(), nb, st())
        torch.cuda.synchronize()
        outs.append((G.cpu(), tags.cpu(), G1.cpu()))
    assert all(torch.equal(x, y) for x, y in zip(outs[0], outs[1]))
    ref = torch.zeros(n_rows, E, dtype=torch.float64)
    ref[0] = 1.0
    use = ids[:n].long()
    ok = (use >= 0) & (use < n_rows) & (use != skip)
    ref.index_add_(0, use[ok], src[:n][ok].double())
    G, tags, G1 = outs[0]
    ref1 = torch.zeros(n_rows, 1, dtype=torch.float64).index_add_(0, use[ok], src[:n][ok][:, :1].double())
    assert float((G1.double() - ref1).abs().max()) < 1e-4
    scale = 1 + torch.zeros(n_rows, E, dtype=torch.float64).index_add_(0, use[ok], src[:n][ok].double().abs())
    assert float(((G.double() - ref).abs() / scale).max()) < 1e-6
    touched = torch.zeros(n_rows, dtype=torch.bool)
    touched[use[ok]] = True
    assert torch.equal(tags == 9, touched)


@pytest.mark.parametrize("H,ndir,B,L", [(128, 1, 100, 9), (128, 2, 70, 6), (64, 2, 70, 6), (32, 1, 33, 5),
                                        (16, 2, 64, 4)])
def test_gru_forward_emits_h_planes(H, ndir, B, L):
    """rg_gru_fwd_dirs_planes: the same final h as rg_gru_fwd_dirs, and its
    bf16 K-planes (the sampled head's operand) bitwise equal to
    rg_head_planes of that h (ragged rows, both directions of a Bidir layer)."""
    g = torch.Generator().manual_seed(H + ndir)
    lens = torch.randint(1, L + 1, (B,), generator=g)
    perm, ls, offs = pack(lens, L)
    T = int(lens.sum())
    k = 1 / H ** 0.5
    Gi = [(torch.randn(T, 3 * H, generator=g) * 0.5).to(dev) for _ in range(ndir)]
    Whh = [((torch.rand(3 * H, H, generator=g) * 2 - 1) * k).to(dev) for _ in range(ndir)]
    bhh = [((torch.rand(3 * H, generator=g) * 2 - 1) * k).to(dev) for _ in range(ndir)]
    HF = ndir * H
    outs = []
    for planes in (False, True):
        hout = torch.zeros(B, HF, device=dev)
        saved = [torch.zeros(5, T, H, device=dev) for _ in range(ndir)]
        args = (C().host_ptr_array(Gi), C().host_ptr_array(Whh), C().host_ptr_array(bhh), C().host_ptr_array(saved),
                ndir, perm.data_ptr(), ls.data_ptr(), offs.data_ptr(), B, H, hout.data_ptr(), HF, 0, T * H)
        hk = torch.zeros(C().call("rg_head_plane_bytes", B, HF), dtype=torch.uint8, device=dev)
        if planes:
            C().call("rg_gru_fwd_dirs_planes", *args, hk.data_ptr(), st())
        else:
            C().call("rg_gru_fwd_dirs", *args, st())
        outs.append((hout, hk))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    ref = torch.zeros_like(outs[1][1])
    C().call("rg_head_planes", outs[1][0].data_ptr(), B, HF, ref.data_ptr(), None, None, None, st())
    torch.cuda.synchronize()
    # rows past B inside the last 32-row block are not written by the GRU: compare the written rows
    n = B // 32 * 32 * HF * 6
    assert torch.equal(outs[1][1][:n], ref[:n])
    if B % 32:
        blk = outs[1][1][n:].view(HF // 16, 3, 2, 32, 16)[..., :B % 32, :]
        rblk = ref[n:].view(HF // 16, 3, 2, 32, 16)[..., :B % 32, :]
        assert torch.equal(blk, rblk)


@pytest.mark.parametrize("n_rows,W,n,n_max,E,zipf", [(1_000_001, 8, 88_000, 90_000, 128, True),
                                                     (53, 3, 700, 700, 4, False), (9001, 2, 1, 64, 64, False),
                                                     (5_000_001, 8, 30_000, 30_000, 256, True)])
def test_shard_dedup_distinct_ids_and_sums(n_rows, W, n, n_max, E, zipf):
    """rg_shard_dedup (the row-sharded table's deduplicated exchange, csrc/
    segsum.hip): the distinct ids sorted (−1 first for invalid tokens), every
    token's index into them, the per-owner counts of dist.owner_counts'
    rules; rg_shard_dedup_grads: per distinct id the sum of its tokens' rows
    (fp64 reference) — bitwise repeatable; Zipf-hot ids whose runs cross many
    64-position blocks."""
    from recommenders.hip.dist import item_shard
    rng = np.random.default_rng(n)
    if zipf:
        ids = (rng.zipf(1.3, size=n) - 1) % n_rows
    else:
        ids = rng.integers(0, n_rows, size=n)
    ids = ids.astype(np.int64)
    raw = ids.copy()
    if n > 10:
        ids[rng.integers(0, n, size=5)] = -1     # invalid tokens (k_token_ids writes -1)
        raw = ids.copy()
        raw[rng.integers(0, n, size=3)] = n_rows + 2   # out of range: counted as -1
        ids = np.where(raw >= n_rows, -1, raw)
    call = C().call
    wb = call("rg_shard_dedup_work_bytes", n_max, E, n_rows)
    work = torch.full((wb,), 0x5A, dtype=torch.uint8, device=dev)   # (no zeroed work buffer needed)
    # an earlier pass on the same work buffer leaves no marks behind
    other = D(torch.from_numpy(rng.integers(0, n_rows, size=n).astype(np.int32)))
    nptr = D(torch.tensor([n], dtype=torch.int32))
    scratch = [torch.empty(n_max, dtype=torch.int32, device=dev) for _ in range(2)]
    call("rg_shard_dedup", other.data_ptr(), nptr.data_ptr(), n_max, n_rows, W, E, scratch[0].data_ptr(),
         scratch[1].data_ptr(), torch.zeros(W, dtype=torch.int32, device=dev).data_ptr(),
         torch.zeros(1, dtype=torch.int32, device=dev).data_ptr(), work.data_ptr(), wb, st())
    tok = D(torch.from_numpy(raw.astype(np.int32)))
    uslot = torch.full((n_max,), -7, dtype=torch.int32, device=dev)
    uids = torch.full((n_max,), -7, dtype=torch.int32, device=dev)
    counts = torch.zeros(W, dtype=torch.int32, device=dev)
    nuniq = torch.zeros(1, dtype=torch.int32, device=dev)
    call("rg_shard_dedup", tok.data_ptr(), nptr.data_ptr(), n_max, n_rows, W, E, uslot.data_ptr(), uids.data_ptr(),
         counts.data_ptr(), nuniq.data_ptr(), work.data_ptr(), wb, st())
    src = torch.from_numpy(rng.standard_normal((n, E)).astype(np.float32))
    srcd = D(src)
    g1 = torch.full((n_max, E), 3.0, device=dev)
    g2 = torch.full((n_max, E), -3.0, device=dev)
    call("rg_shard_dedup_grads", srcd.data_ptr(), E, n_max, n_rows, g1.data_ptr(), work.data_ptr(), wb, st())
    call("rg_shard_dedup_grads", srcd.data_ptr(), E, n_max, n_rows, g2.data_ptr(), work.data_ptr(), wb, st())
    torch.cuda.synchronize()
    U = int(nuniq.item())
    exp_u = np.unique(ids)
    assert U == exp_u.size
    np.testing.assert_array_equal(uids[:U].cpu().numpy(), exp_u)
    sl = uslot[:n].cpu().numpy()
    np.testing.assert_array_equal(exp_u[sl], ids)
    seen = np.zeros(W, dtype=np.int64)
    for x in exp_u:
        seen[0 if x < 0 else next(r for r in range(W) if item_shard(n_rows, W, r)[0] <= x < item_shard(n_rows, W, r)[1])] += 1
    np.testing.assert_array_equal(counts.cpu().numpy(), seen)
    ref = np.zeros((U, E))
    np.add.at(ref, sl, src.numpy().astype(np.float64))
    got = g1[:U].cpu().numpy()
    scale = np.maximum(1.0, np.sqrt(np.bincount(sl, minlength=U)))[:, None]
    assert (np.abs(got - ref) <= 1e-5 * scale).all()
    assert torch.equal(g1[:U], g2[:U])   # fixed order: bitwise repeatable, stored not added


@pytest.mark.parametrize("n_rows,B,L,packed,bad", [(1_000_001, 4096, 50, True, True), (53, 37, 9, False, False),
                                                   (9001, 64, 20, True, False), (5_000_001, 512, 50, True, True)])
def test_shard_dedup_ids_equals_the_device_dedup(n_rows, B, L, packed, bad):
    """rg_shard_dedup_ids (the distinct ids from the host batch, dist.distinct_ids)
    against rg_token_ids + rg_shard_dedup on the same packed batch: tok_id,
    uslot, the distinct ids, the error flag and rg_shard_dedup_grads' per-id
    sums from the work pairs — all bitwise; the map is reused across batches
    without clearing."""
    from recommenders.hip.dist import distinct_ids
    rng = np.random.default_rng(n_rows + B)
    call = C().call
    E = 64
    for rep in range(2):
        s = ((rng.zipf(1.3, size=(B, L)) - 1) % n_rows).astype(np.int64)
        if bad:
            s[rng.integers(0, B, 4), rng.integers(0, 3, 4)] = -1
            s[rng.integers(0, B, 2), 0] = n_rows + 5
        lens = rng.integers(0, L + 2, size=B).astype(np.int64)
        sd, ld = D(torch.from_numpy(s)), D(torch.from_numpy(lens))
        perm = torch.empty(B, dtype=torch.int32, device=dev)
        lsort = torch.empty(B, dtype=torch.int32, device=dev)
        offs = torch.empty(B + 1, dtype=torch.int32, device=dev)
        call("rg_pack", ld.data_ptr(), B, L, 0 if packed else 1, perm.data_ptr(), lsort.data_ptr(), offs.data_ptr(),
             st())
        nptr = offs.data_ptr() + 4 * B
        n_max = B * L
        wb = call("rg_shard_dedup_work_bytes", n_max, E, n_rows)
        outs = []
        for host in (False, True):
            work = torch.full((wb,), 0x5A, dtype=torch.uint8, device=dev)
            tok = torch.full((n_max,), -9, dtype=torch.int32, device=dev)
            uslot = torch.full((n_max,), -9, dtype=torch.int32, device=dev)
            uids = torch.full((n_max,), -9, dtype=torch.int32, device=dev)
            err = torch.zeros(1, dtype=torch.int32, device=dev)
            if host:
                u = distinct_ids(s, lens, L, packed, n_rows)
                uids[:u.size] = D(torch.from_numpy(u))
                if rep == 0:
                    dd_map = torch.full((n_rows + 1,), 0x7FFF, dtype=torch.int32, device=dev)
                call("rg_shard_dedup_ids", sd.data_ptr(), B, L, perm.data_ptr(), lsort.data_ptr(), offs.data_ptr(),
                     nptr, n_max, n_rows, uids.data_ptr(), int(u.size), dd_map.data_ptr(), tok.data_ptr(),
                     uslot.data_ptr(), err.data_ptr(), E, work.data_ptr(), wb, st())
                U = int(u.size)
            else:
                nuniq = torch.zeros(1, dtype=torch.int32, device=dev)
                call("rg_token_ids", sd.data_ptr(), B, L, perm.data_ptr(), lsort.data_ptr(), offs.data_ptr(), n_rows,
                     tok.data_ptr(), err.data_ptr(), st())
                call("rg_shard_dedup", tok.data_ptr(), nptr, n_max, n_rows, 4, E, uslot.data_ptr(), uids.data_ptr(),
                     torch.zeros(4, dtype=torch.int32, device=dev).data_ptr(), nuniq.data_ptr(), work.data_ptr(), wb,
                     st())
                U = int(nuniq.item())
            T = int(offs[B].item())
            src = D(torch.from_numpy(rng.standard_normal((n_max, E)).astype(np.float32))) if not host else outs[0][5]
            g = torch.full((n_max, E), 3.0, device=dev)
            call("rg_shard_dedup_grads", src.data_ptr(), E, n_max, n_rows, g.data_ptr(), work.data_ptr(), wb, st())
            torch.cuda.synchronize()
            outs.append((tok[:T].clone(), uslot[:T].clone(), uids[:U].clone(), int(err.item()), g[:U].clone(), src))
        (t0, s0, u0, e0, g0, _), (t1, s1, u1, e1, g1, _) = outs
        assert torch.equal(t0, t1) and torch.equal(s0, s1) and torch.equal(u0, u1) and e0 == e1
        assert e1 == (1 if bad else 0)
        assert torch.equal(g0, g1)


@pytest.mark.parametrize("nplanes", [3, 1])
@pytest.mark.parametrize("A,HF,nh", [(20011, 128, 3), (777, 256, 2), (1000, 64, 3), (4096, 32, 1)])
def test_qcomb_equals_weighted_sum_planes_norm(A, HF, nh, nplanes):
    """rg_qcomb (the SMORL target's combined Q head in one pass) against the
    separate kernels it replaces: W_c / b_c bitwise rg_weighted_sum's, the
    K-planes (all three, or plane 0 only for the one-product screening) and
    padded bias bitwise rg_head_planes', the max row norm within fp32
    rounding of rg_row_norm_max's (another summation order) and of fp64."""
    call = C().call
    g = torch.Generator().manual_seed(A + HF)
    Ws = [D(torch.randn(A, HF, generator=g) * 0.1) for _ in range(nh)]
    bs = [D(torch.randn(A, generator=g) * 0.1) for _ in range(nh)]
    wts = [1.0, 0.5, 2.0][:nh]
    hw = C().host_floats(wts)
    Wc, bc = torch.empty(A, HF, device=dev), torch.empty(A, device=dev)
    pk = torch.empty(call("rg_head_plane_bytes", A, HF), dtype=torch.uint8, device=dev)
    Ap = (A + 31) // 32 * 32
    bp = torch.empty(Ap, device=dev)
    wn = torch.full((1,), 7.0, device=dev)
    call("rg_qcomb", C().host_ptr_array(Ws), C().host_ptr_array(bs), hw, nh, A, HF, nplanes, Wc.data_ptr(),
         bc.data_ptr(), pk.data_ptr(), bp.data_ptr(), wn.data_ptr(), st())
    Wr, br = torch.empty_like(Wc), torch.empty_like(bc)
    call("rg_weighted_sum", C().host_ptr_array(Ws), hw, nh, A * HF, Wr.data_ptr(), st())
    call("rg_weighted_sum", C().host_ptr_array(bs), hw, nh, A, br.data_ptr(), st())
    pk2 = torch.empty_like(pk)
    bp2 = torch.empty_like(bp)
    call("rg_head_planes", Wr.data_ptr(), A, HF, pk2.data_ptr(), None, br.data_ptr(), bp2.data_ptr(), st())
    wn2 = torch.zeros(1, device=dev)
    call("rg_row_norm_max", Wr.data_ptr(), A, HF, wn2.data_ptr(), st())
    torch.cuda.synchronize()
    assert torch.equal(Wc, Wr) and torch.equal(bc, br)
    planes = lambda t: t.view(-1, 3, 64, 16)[:, :nplanes]   # noqa: E731  (plane p: entries 64p .. 64p + 63 of each triple)
    assert torch.equal(planes(pk), planes(pk2)) and torch.equal(bp, bp2)
    ref = float(Wr.double().norm(dim=1).max())
    assert abs(float(wn) - float(wn2)) <= 2e-6 * ref and abs(float(wn) - ref) <= 2e-6 * ref


@pytest.mark.parametrize("T,W", [(4096, 8), (4096, 1), (3001, 3), (20000, 2), (1, 8), (0, 4)])
def test_shard_route_is_stable_partition_by_owner(T, W):
    """rg_shard_route (the sharded sampled head's per-row target exchange,
    csrc/emb_shard.hip): counts per owner, and every row's send slot — rows
    grouped by owner (invalid ids with rank 0), in row order within an owner."""
    from recommenders.hip.dist import item_shard
    n_rows = 90001
    rng = np.random.default_rng(T + W)
    ids = rng.integers(0, n_rows, size=max(T, 1)).astype(np.int32)
    if T > 10:
        ids[rng.integers(0, T, size=7)] = -1
    call = C().call
    tok = D(torch.from_numpy(ids))
    nptr = D(torch.tensor([T], dtype=torch.int32))
    slot = torch.full((max(T, 1),), -5, dtype=torch.int32, device=dev)
    send = torch.full((max(T, 1),), -5, dtype=torch.int32, device=dev)
    counts = torch.full((W,), -5, dtype=torch.int32, device=dev)
    call("rg_shard_route", tok.data_ptr(), nptr.data_ptr(), n_rows, W, slot.data_ptr(), send.data_ptr(),
         counts.data_ptr(), st())
    torch.cuda.synchronize()
    ids = ids[:T]
    own = np.array([0 if x < 0 else next(r for r in range(W) if item_shard(n_rows, W, r)[0] <= x < item_shard(n_rows, W, r)[1])
                    for x in ids], dtype=np.int64)
    order = np.argsort(own, kind="stable")
    exp_slot = np.empty(T, dtype=np.int64)
    exp_slot[order] = np.arange(T)
    np.testing.assert_array_equal(counts.cpu().numpy(), np.bincount(own, minlength=W))
    np.testing.assert_array_equal(slot[:T].cpu().numpy(), exp_slot)
    np.testing.assert_array_equal(send[:T].cpu().numpy(), ids[order])


@pytest.mark.parametrize("terms", [6, 9])
@pytest.mark.parametrize("M,N,K,bk", [(85003, 384, 128, 1), (300, 128, 384, 0), (129, 768, 256, 1), (4100, 64, 96, 0),
                                      (7, 32, 32, 1), (1000, 256, 384, 0)])
def test_gemm_x6_split_bf16(terms, M, N, K, bk):
    """rg_gemm_x6 (split-bf16 trunk GEMM: Gi = X·W_ihᵀ + b with B k-contiguous,
    dX = dGi·W_ih with B n-contiguous): against fp64, within 2× the native
    fp32 MFMA kernel's own error (rg_gemm_f32) plus fp32 rounding of the
    output; device-side row count, partial tiles, rows past M untouched."""
    g = torch.Generator().manual_seed(5 + M + K)
    A = torch.randn(M, K, generator=g)
    Bnk = torch.randn(N, K, generator=g) * 0.1
    bias = torch.randn(N, generator=g) if bk else None
    ref = A.double() @ Bnk.double().t() + (bias.double() if bk else 0)
    Ad = D(A)
    Bd = D(Bnk) if bk else D(Bnk.t().contiguous())
    ldb = K if bk else N
    Mdev = D(torch.tensor([M], dtype=torch.int32))
    out = torch.full((M + 5, N), float("nan"), device=dev)
    C().call("rg_gemm_x6", Ad.data_ptr(), K, Bd.data_ptr(), ldb, bk, out.data_ptr(), N,
             D(bias).data_ptr() if bk else None, M + 300, Mdev.data_ptr(), N, K, terms, st())
    nat = torch.full((M, N), float("nan"), device=dev)
    C().call("rg_gemm_f32", Ad.data_ptr(), K, 1, Bd.data_ptr(), 1 if bk else N, K if bk else 1, nat.data_ptr(), N,
             D(bias).data_ptr() if bk else None, M, None, N, K, None, 1, st())
    torch.cuda.synchronize()
    assert torch.isnan(out[M:]).all()
    e_x6 = (out[:M].cpu().double() - ref).abs().max().item()
    e_nat = (nat.cpu().double() - ref).abs().max().item()
    ulp = ref.abs().max().item() * 2.0 ** -24
    assert e_x6 <= 2 * e_nat + 2 * ulp, (e_x6, e_nat, ulp)


@pytest.mark.parametrize("terms", [6, 9])
@pytest.mark.parametrize("M,N,K,splits,ak,bk", [(4096, 256, 2048, 8, 1, 0), (2048, 256, 4096, 16, 0, 0),
                                                (300, 128, 320, 3, 1, 1), (130, 64, 96, 5, 0, 1),
                                                (512, 32, 512, 1, 0, 0)])
def test_gemm_x6_split_k(terms, M, N, K, splits, ak, bk):
    """rg_gemm_x6_sk (the sampled head's dh = dZ·W_neg, A k-contiguous, and
    dW_neg = dZᵀ·h, A m-contiguous; split-K slabs, a ragged last chunk, more
    splits than stages): the slabs' sum against fp64 within 2× the native
    fp32 split-K kernel's error (rg_gemm_f32 with the same splits)."""
    g = torch.Generator().manual_seed(7 + M + K + splits)
    A = torch.randn(M, K, generator=g)
    Bnk = torch.randn(N, K, generator=g) * 0.1
    ref = A.double() @ Bnk.double().t()
    Ad = D(A) if ak else D(A.t().contiguous())
    lda = K if ak else M
    Bd = D(Bnk) if bk else D(Bnk.t().contiguous())
    ldb = K if bk else N
    out = torch.full((splits, M, N), float("nan"), device=dev)
    C().call("rg_gemm_x6_sk", Ad.data_ptr(), lda, ak, Bd.data_ptr(), ldb, bk, out.data_ptr(), N, M * N, M, N, K,
             splits, terms, st())
    nat = torch.full((splits, M, N), float("nan"), device=dev)
    C().call("rg_gemm_f32", Ad.data_ptr(), K if ak else 1, 1 if ak else M, Bd.data_ptr(), 1 if bk else N,
             K if bk else 1, nat.data_ptr(), N, None, M, None, N, K, None, splits, st())
    torch.cuda.synchronize()
    kchunk = (K // 32 + splits - 1) // splits * 32
    used = (K + kchunk - 1) // kchunk   # slabs past the last k chunk are zero
    got = out[:used].sum(0).cpu().double()
    assert torch.count_nonzero(out[used:].nan_to_num(1.0)) == 0
    e_x6 = (got - ref).abs().max().item()
    e_nat = (nat.sum(0).cpu().double() - ref).abs().max().item()
    ulp = ref.abs().max().item() * 2.0 ** -24
    assert e_x6 <= 2 * e_nat + 2 * splits * ulp, (e_x6, e_nat, ulp)


@pytest.mark.parametrize("terms", [6, 9])
@pytest.mark.parametrize("M,N,T,splits", [(384, 128, 5000, 16), (384, 256, 3000, 7), (192, 64, 3000, 128),
                                          (96, 32, 777, 3), (384, 128, 85000, 128)])
def test_wgrad_x6_split_bf16(terms, M, N, T, splits):
    """rg_wgrad_x6 (split-bf16 dW = Gᵀ·X and db = Σ G over device-counted
    tokens, token-split slabs): against fp64, within 2× rg_wgrad's error."""
    g = torch.Generator().manual_seed(9 + T)
    G = torch.randn(T + 40, M, generator=g)
    X = torch.randn(T + 40, N, generator=g)
    Tdev = D(torch.tensor([T], dtype=torch.int32))
    out = {}
    for name in ("rg_wgrad_x6", "rg_wgrad"):
        dw = torch.full((splits, M, N), float("nan"), device=dev)
        db = torch.full((splits, M), float("nan"), device=dev)
        extra = (terms,) if name.endswith("x6") else ()
        C().call(name, D(G).data_ptr(), M, D(X).data_ptr(), N, T + 40, Tdev.data_ptr(), splits, dw.data_ptr(),
                 db.data_ptr(), *extra, st())
        out[name] = (dw.sum(0).cpu().double(), db.sum(0).cpu().double())
    ref_w = G[:T].double().t() @ X[:T].double()
    ref_b = G[:T].double().sum(0)
    e_w = {k: (v[0] - ref_w).abs().max().item() for k, v in out.items()}
    e_b = {k: (v[1] - ref_b).abs().max().item() for k, v in out.items()}
    assert e_w["rg_wgrad_x6"] <= 2 * e_w["rg_wgrad"] + 1e-6 * T ** 0.5, e_w
    assert e_b["rg_wgrad_x6"] <= 2 * e_b["rg_wgrad"] + 1e-6 * T ** 0.5, e_b
