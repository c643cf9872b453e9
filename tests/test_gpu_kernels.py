"""GPU parity of the individual libctr_hip.so kernels against the oracle / numpy.

Tolerances (written per test): integer / index work bit-exact; fp32 sums within 1e-5
relative of an fp64 reference (the north-star bar), with an absolute floor where the
quantity is a difference of nearly equal terms.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import ctr_oracle as O

pytestmark = pytest.mark.gpu


def _hip():
    from rl_ctr_prediction_amd import hip_ops
    return hip_ops


def _ids(rng, B, F, V, hot=True, layout="uniform"):
    """uniform: every column draws from [0, V) (column ranges overlap: the column plan's
    binary-search merge and segment launches); fields: column f draws from a range of its
    own, [f*card, (f+1)*card) with Zipf-skewed values (the CTR layout: the merge writes the
    whole plan)."""
    if layout == "fields":
        card = V // F
        x = np.minimum(rng.zipf(1.2, size=(B, F)) - 1, card - 1) + np.arange(F) * card
        return x
    x = rng.integers(0, V, size=(B, F))
    if hot and B > 1 and F > 2:
        x[:, 0] = min(7, V - 1)
        x[: B // 2, 1] = min(3, V - 1)
    return x


# ----------------------------------------------------------------- sparse plan ------
@pytest.mark.parametrize("B,F,V", [(1, 1, 1), (3, 5, 2), (64, 26, 1000), (257, 13, 50),
                                   (4096, 26, 1_000_000), (1000, 39, 1508), (33, 16, 7),
                                   (8192, 26, 10_000_000), (20165, 26, 2),
                                   (65536, 26, 40_000_000), (777, 22, 2**31 - 1)])
@pytest.mark.parametrize("dtype", [torch.int64, torch.int32])
@pytest.mark.parametrize("layout", ["uniform", "fields"])
@pytest.mark.parametrize("cols", [True, False])
def test_sparse_plan_bit_exact(cuda, B, F, V, dtype, layout, cols):
    """cols: [B, F] ids (the column plan, ctr_sparse_plan_build_cols: per-column LDS sorts +
    merge; B > 8192 falls back to the LSD plan); else the flat ids
    (the LSD plan). Both bit-exact vs numpy's stable argsort / unique."""
    if layout == "fields" and V < 2 * F:
        pytest.skip("fields need V >= 2F")
    H = _hip()
    rng = np.random.default_rng(B * 31 + F)
    x = _ids(rng, B, F, V, layout=layout)
    xt = torch.tensor(x, dtype=dtype, device=cuda)
    plan = H.SparsePlanBuffers(B * F, cuda).build(xt if cols else xt.reshape(-1), V)
    order, rows, pos_seg, uniq, off = O.sparse_plan(x)
    U = plan.num_unique_host()
    assert U == uniq.size
    np.testing.assert_array_equal(plan.sorted_slots.cpu().numpy()[: B * F], order)
    np.testing.assert_array_equal(plan.sorted_rows.cpu().numpy()[: B * F], rows)
    np.testing.assert_array_equal(plan.pos_seg.cpu().numpy()[: B * F], pos_seg)
    np.testing.assert_array_equal(plan.unique_rows.cpu().numpy()[:U], uniq)
    np.testing.assert_array_equal(plan.seg_offsets.cpu().numpy()[: U + 1], off)


def test_sparse_plan_rebuilds_and_graph_replay(cuda):
    """The same plan buffers rebuilt for batches of both layouts in turn (the column plan's
    merge decides per build whether the segment launches run), eagerly and as a replayed
    HIP graph, stay bit-exact; no error flag."""
    H = _hip()
    rng = np.random.default_rng(5)
    B, F, V = 4096, 26, 1_000_000
    xs = [torch.tensor(_ids(rng, B, F, V, layout=("fields", "uniform")[j % 2]), device=cuda)
          for j in range(4)]
    ids = torch.empty_like(xs[0])
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    plan = H.SparsePlanBuffers(B * F, cuda)
    plan.build(xs[0], V, err_flag=err)  # sizes the scratch
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ids.copy_(xs[0])
        with torch.cuda.graph(g, stream=s):
            plan.build(ids, V, err_flag=err)
    torch.cuda.current_stream().wait_stream(s)
    for i, x in enumerate(xs * 2):
        if i % 2:
            plan.build(x, V, err_flag=err)
        else:
            ids.copy_(x)
            g.replay()
        torch.cuda.synchronize()
        order, rows, pos_seg, uniq, off = O.sparse_plan(x.cpu().numpy())
        U = plan.num_unique_host()
        assert U == uniq.size, i
        np.testing.assert_array_equal(plan.sorted_slots.cpu().numpy()[: B * F], order)
        np.testing.assert_array_equal(plan.pos_seg.cpu().numpy()[: B * F], pos_seg)
        np.testing.assert_array_equal(plan.seg_offsets.cpu().numpy()[: U + 1], off)
    assert int(err.item()) == 0


@pytest.mark.parametrize("layout", ["uniform", "fields"])
def test_sparse_plan_invalid_ids(cuda, layout):
    """Ids outside [0, V) raise the index flag and are grouped as row 0 by both builds
    (nn.Embedding raises before any update; the trainers check the flag)."""
    H = _hip()
    rng = np.random.default_rng(9)
    B, F, V = 1000, 26, 100_000
    x = _ids(rng, B, F, V, layout=layout)
    x[5, 3], x[700, 20], x[999, 25] = -1, V, V + 77
    xt = torch.tensor(x, device=cuda)
    out = []
    for ids in (xt, xt.reshape(-1)):
        err = torch.zeros(1, dtype=torch.int32, device=cuda)
        plan = H.SparsePlanBuffers(B * F, cuda).build(ids, V, err_flag=err)
        assert int(err.item()) & 1
        U = plan.num_unique_host()
        out.append([t.cpu().numpy().copy() for t in (plan.sorted_slots, plan.sorted_rows,
                    plan.pos_seg)] + [plan.unique_rows[:U].cpu().numpy(),
                                      plan.seg_offsets[:U + 1].cpu().numpy()])
    xf = np.where((x < 0) | (x >= V), 0, x)
    ref = O.sparse_plan(xf)
    for got in out:
        for a, b in zip(got, ref):
            np.testing.assert_array_equal(a[:b.size], b)


def test_sparse_plan_empty(cuda):
    H = _hip()
    plan = H.SparsePlanBuffers(0, cuda).build(torch.zeros(0, 26, dtype=torch.int64, device=cuda), 10)
    assert plan.num_unique_host() == 0


# --------------------------------------------------------------- segmented sums -----
@pytest.mark.parametrize("K", [1, 10, 16, 64, 128])
@pytest.mark.parametrize("S,V", [(1, 1), (15, 3), (16, 1), (17, 1), (1000, 10), (5000, 4000),
                                 (20000, 60)])
def test_segment_sum_rows(cuda, K, S, V):
    H = _hip()
    rng = np.random.default_rng(S + K)
    keys = rng.integers(0, V, size=S)
    keys[: S // 3] = 0  # one hot row spanning many 16-position chunks
    vals = rng.standard_normal((S, K)).astype(np.float32)
    lin = rng.standard_normal(S).astype(np.float32)
    plan = H.SparsePlanBuffers(S, cuda).build(torch.tensor(keys, dtype=torch.int32, device=cuda), V)
    rowmap = torch.full((V,), -1, dtype=torch.int32, device=cuda)
    tv, tl = torch.tensor(vals, device=cuda), torch.tensor(lin, device=cuda)
    out, out_lin = H.segment_sum_rows(plan, tv, tl, rowmap=rowmap)
    U = plan.num_unique_host()
    uniq = np.unique(keys)
    ref = np.zeros((V, K))
    np.add.at(ref, keys, vals.astype(np.float64))
    refl = np.zeros(V)
    np.add.at(refl, keys, lin.astype(np.float64))
    got = out[:U].cpu().numpy()
    scale = np.zeros((V, K))
    np.add.at(scale, keys, np.abs(vals.astype(np.float64)))
    np.testing.assert_allclose(got, ref[uniq], rtol=1e-5, atol=1e-6 * (1 + scale[uniq]).max())
    np.testing.assert_allclose(out_lin[:U].cpu().numpy(), refl[uniq], rtol=1e-5, atol=1e-4)
    rm = rowmap.cpu().numpy()
    assert (rm[uniq] == np.arange(U)).all() and (np.delete(rm, uniq) == -1).all()
    # deterministic: a second run is bitwise identical
    out2, out_lin2 = H.segment_sum_rows(plan, tv, tl)
    assert torch.equal(out[:U], out2[:U]) and torch.equal(out_lin[:U], out_lin2[:U])


# ------------------------------------------------------------------- FM forward -----
@pytest.mark.parametrize("K", [10, 16, 64, 128])
@pytest.mark.parametrize("F", [1, 8, 26, 39, 70])
def test_fm_forward_vs_oracle(cuda, K, F):
    H = _hip()
    V, B = 500, 67
    rng = np.random.default_rng(K * 100 + F)
    E = (rng.standard_normal((V, K)) * 0.1).astype(np.float32)
    w = (rng.standard_normal((V, 1)) * 0.1).astype(np.float32)
    b = np.array([0.05], np.float32)
    x = _ids(rng, B, F, V)
    y = (rng.random(B) < 0.3).astype(np.float32)
    params = {"feature_embedding.weight": torch.tensor(E), "linear.weight": torch.tensor(w),
              "bias": torch.tensor(b)}
    z_ref = O.fm_logit(params, torch.tensor(x)).reshape(-1).double()
    d = lambda a: torch.tensor(a, device=cuda)  # noqa: E731
    r = H.fm_forward(d(x), d(E), d(w), d(b), want_sum=True, want_emb=True, labels=d(y))
    zt = r.z.cpu().double()
    e = E[x]
    # the FM term is a difference of sums: its rounding error scales with the magnitudes
    # summed (sum_k (s_k^2 + q_k) + sum_f |w|), not with |z|
    mag = 0.5 * ((e.sum(1) ** 2).sum(1) + (e ** 2).sum((1, 2))) + np.abs(w[x]).sum((1, 2)) + 0.05
    assert (np.abs(zt.numpy() - z_ref.numpy()) <= 1e-5 * np.abs(z_ref.numpy()) + 1e-6 * mag).all()
    np.testing.assert_allclose(r.sum_e.cpu().numpy(), e.sum(1), rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(r.emb_out.cpu().numpy(), e.reshape(B, -1))
    p = torch.sigmoid(z_ref.float())
    np.testing.assert_allclose(r.p.cpu().numpy(), p.numpy(), rtol=1e-5, atol=1e-7)


def test_fm_forward_saturated_gradient_is_exactly_zero(cuda, golden):
    H = _hip()
    g = golden("g_bce.npz")
    z, y = torch.tensor(g["z"], device=cuda), torch.tensor(g["y"], device=cuda)
    p, loss, gz = H.bce_sigmoid(z, y)
    np.testing.assert_allclose(p.cpu().numpy(), g["p"], rtol=1e-6, atol=0)
    ref_gz = g["gz"]
    zero = ref_gz == 0
    assert (gz.cpu().numpy()[zero] == 0).all(), "saturated sigmoid must give a 0 gradient"
    np.testing.assert_allclose(gz.cpu().numpy(), ref_gz, rtol=2e-5, atol=0)
    assert loss.mean().item() == pytest.approx(float(g["loss"]), rel=1e-5)


def test_out_of_range_ids_flag_not_fault(cuda):
    H = _hip()
    V, K = 100, 16
    E = torch.randn(V, K, device=cuda)
    w = torch.randn(V, 1, device=cuda)
    b = torch.zeros(1, device=cuda)
    x = torch.randint(0, V, (8, 26), device=cuda)
    x[3, 4] = V + 5
    x[5, 0] = -1
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    H.fm_forward(x, E, w, b, err_flag=err)
    with pytest.raises(IndexError):
        H.check_index_error(err)
    H.check_index_error(err)  # flag was cleared


# ------------------------------------------------------------------------- GEMM -----
_ALGO = {"exact": 1, "split": 2}  # enum ctr_gemm_algo (hip_ops.GEMM_EXACT_F32 / _SPLIT_BF16)


def test_gemm_split_bf16_accuracy(cuda):
    """The split-bf16 GEMM is at least as accurate as the exact-fp32 one: on the DeepFM
    shapes its worst error against fp64, relative to the L1 bound, is no larger than the
    fp32 kernel's (its main accumulator rounds once per 16 k, the fp32 MFMA chain 8 times;
    measured ~0.3-0.45x), and both are far under the 1e-5 bar."""
    H = _hip()
    g = torch.Generator().manual_seed(5)
    for (M, N, K, ta, tb) in ((8192, 300, 1664, False, True), (300, 1664, 8192, True, False),
                              (8192, 1664, 300, False, False)):
        A = torch.randn(M, K, generator=g) * 0.1
        Bm = torch.randn(K, N, generator=g)
        a = (A.t() if ta else A).contiguous().to(cuda)
        b = (Bm.t() if tb else Bm).contiguous().to(cuda)
        ref = A.double() @ Bm.double()
        bound = A.double().abs() @ Bm.double().abs()
        err = {}
        for name, algo in _ALGO.items():
            C = H.gemm(a, b, ta, tb, algo=algo).cpu().double()
            err[name] = ((C - ref).abs() / bound).max().item()
        assert err["split"] < 1e-6, err
        assert err["split"] <= err["exact"], (M, N, K, err)
@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (7, 5, 3), (64, 64, 32), (130, 70, 33),
                                   (300, 1664, 8192), (8192, 300, 1664), (8192, 1664, 300),
                                   (512, 200, 300), (4, 1024, 741)])
@pytest.mark.parametrize("algo", ["exact", "split"])
def test_gemm_vs_fp64(cuda, ta, tb, M, N, K, algo):
    H = _hip()
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    A = torch.randn(M, K, generator=g)
    Bm = torch.randn(K, N, generator=g)
    a = (A.t() if ta else A).contiguous().to(cuda)
    b = (Bm.t() if tb else Bm).contiguous().to(cuda)
    C = H.gemm(a, b, ta, tb, algo=_ALGO[algo]).cpu().double()
    ref = A.double() @ Bm.double()
    bound = (A.double().abs() @ Bm.double().abs())
    # fp32 accumulation (exact-fp32 MFMA = a k-ordered fmaf chain; split-bf16: products to
    # 2^-23 relative, fp32 accumulation): error grows ~sqrt(K)
    tol = 1e-6 * max(1.0, (K / 1024) ** 0.5)
    assert ((C - ref).abs() <= tol * bound + 1e-30).all()


def _gemm_tilings(n_tiles, algo_name):
    return [(algo_name, t) for t in range(n_tiles)]


# every compiled tiling of csrc/gemm.hip (kTiles) and csrc/gemm_sb16.hip (kSb16)
@pytest.mark.parametrize("algo,tile", _gemm_tilings(10, "exact") + _gemm_tilings(8, "split"))
def test_gemm_every_tiling(cuda, algo, tile, monkeypatch):
    """Force each tiling (and split-K) on shapes with M/N edges and K tails, both the float4
    path (extents % 4 == 0) and the scalar path, every transpose: fp32 parity vs fp64."""
    H = _hip()
    g = torch.Generator().manual_seed(tile)
    for splits in (1, 3):
        monkeypatch.setenv("CTR_GEMM_CFG", f"{tile},{splits}")
        for (M, N, K) in ((333, 452, 1060), (97, 451, 259)):
            A = torch.randn(M, K, generator=g)
            Bm = torch.randn(K, N, generator=g)
            ref = A.double() @ Bm.double()
            bound = A.double().abs() @ Bm.double().abs()
            for ta in (False, True):
                for tb in (False, True):
                    a = (A.t() if ta else A).contiguous().to(cuda)
                    b = (Bm.t() if tb else Bm).contiguous().to(cuda)
                    C = H.gemm(a, b, ta, tb, algo=_ALGO[algo]).cpu().double()
                    bad = (C - ref).abs() > 2e-6 * bound + 1e-30
                    assert not bad.any(), (tile, splits, M, N, K, ta, tb, int(bad.sum()))
        bias = torch.randn(452, generator=g)
        A = torch.randn(333, 1060, generator=g)
        W = torch.randn(452, 1060, generator=g)
        y = H.gemm(A.to(cuda), W.to(cuda), False, True, epi=H.EPI_BIAS_RELU, bias=bias.to(cuda),
                   algo=_ALGO[algo]).cpu().double()
        r = (A.double() @ W.double().t() + bias.double()).clamp(min=0)
        np.testing.assert_allclose(y.numpy(), r.numpy(), rtol=1e-5, atol=1e-4)


def test_gemm_epilogues(cuda):
    H = _hip()
    g = torch.Generator().manual_seed(0)
    M, N, K = 512, 300, 128
    A, W, bias = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g), torch.randn(N, generator=g)
    d = lambda t: t.contiguous().to(cuda)  # noqa: E731
    ref = (A.double() @ W.double().t() + bias.double())
    y = H.linear(d(A), d(W), d(bias)).cpu().double()
    np.testing.assert_allclose(y.numpy(), ref.numpy(), rtol=1e-5, atol=1e-4)
    y = H.linear(d(A), d(W), d(bias), relu=True).cpu().double()
    np.testing.assert_allclose(y.numpy(), ref.clamp(min=0).numpy(), rtol=1e-5, atol=1e-4)
    yd = H.linear(d(A), d(W), d(bias), relu=True, drop_p=0.2, seed=123).cpu().double()
    pos = ref > 1e-3
    kept = (yd[pos] != 0)
    frac = kept.double().mean().item()
    assert 0.78 < frac < 0.82, frac  # Bernoulli(0.8) keep rate
    np.testing.assert_allclose(yd[pos][kept].numpy(), (ref[pos][kept] * 1.25).numpy(), rtol=1e-5,
                               atol=1e-4)
    yd2 = H.linear(d(A), d(W), d(bias), relu=True, drop_p=0.2, seed=123).cpu().double()
    assert torch.equal(yd, yd2)  # stateless mask: same (seed, offset) -> same mask
    aux = d(yd.float())
    gm = H.gemm(d(A), d(W), False, True, epi=H.EPI_GRAD_MASK, aux=aux, scale=1.25).cpu().double()
    refm = torch.where(yd > 0, (A.double() @ W.double().t()) * 1.25, torch.zeros_like(yd))
    np.testing.assert_allclose(gm.numpy(), refm.numpy(), rtol=1e-5, atol=1e-4)


def test_reductions(cuda):
    H = _hip()
    g = torch.Generator().manual_seed(1)
    for M, N in [(1, 1), (8192, 300), (4096, 1), (7, 129), (100000, 3)]:
        X = torch.randn(M, N, generator=g)
        w = torch.randn(M, generator=g)
        c = H.colsum(X.to(cuda), w.to(cuda), scale=0.5).cpu().double()
        ref = 0.5 * (w.double()[:, None] * X.double()).sum(0)
        np.testing.assert_allclose(c.numpy(), ref.numpy(), rtol=1e-5, atol=1e-5 * M ** 0.5)
        s = H.tensor_sum(X.reshape(-1).contiguous().to(cuda), scale=2.0).item()
        assert s == pytest.approx(2.0 * X.double().sum().item(), rel=1e-5, abs=1e-4 * (M * N) ** 0.5)


# ------------------------------------------------------------------------- Adam -----
def _torch_adam_ref(p0, grads, lr, wd, steps):
    p = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([p], lr=lr, weight_decay=wd)
    for g in grads[:steps]:
        p.grad = g.clone()
        opt.step()
    st = opt.state[p]
    return p.detach(), st["exp_avg"], st["exp_avg_sq"]


def test_adam_dense_vs_torch_cpu(cuda):
    H = _hip()
    g = torch.Generator().manual_seed(2)
    n = 100003
    p0 = torch.randn(n, generator=g) * 0.1
    grads = [torch.randn(n, generator=g) * 1e-3 for _ in range(3)]
    p, m, v = p0.clone().to(cuda), torch.zeros(n, device=cuda), torch.zeros(n, device=cuda)
    for t in range(3):
        H.adam_dense(p, grads[t].to(cuda), m, v, t + 1, 1e-3, weight_decay=1e-5)
        pr, mr, vr = _torch_adam_ref(p0, grads, 1e-3, 1e-5, t + 1)
        if t == 0:  # same inputs: torch's FMA forms reproduced bit-exactly
            np.testing.assert_array_equal(m.cpu().numpy(), mr.numpy())
            np.testing.assert_array_equal(v.cpu().numpy(), vr.numpy())
        else:  # later steps see p (through wd*p) that differs by a few ulps of the step
            np.testing.assert_allclose(m.cpu().numpy(), mr.numpy(), rtol=1e-6, atol=1e-12)
            np.testing.assert_allclose(v.cpu().numpy(), vr.numpy(), rtol=1e-6, atol=1e-18)
        np.testing.assert_allclose(p.cpu().numpy(), pr.numpy(), rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("K", [10, 16, 64])
def test_adam_embedding_dense_semantics(cuda, K):
    """Touched rows get their gradient, untouched rows still move (g = wd*p), as with a
    dense nn.Embedding gradient + torch.optim.Adam."""
    H = _hip()
    g = torch.Generator().manual_seed(K)
    V = 3001
    E0 = torch.randn(V, K, generator=g) * 0.1
    w0 = torch.randn(V, 1, generator=g) * 0.1
    touched = torch.unique(torch.randint(0, V, (700,), generator=g)).to(torch.int32)
    U = touched.numel()
    gr = torch.randn(U, K, generator=g) * 1e-2
    gl = torch.randn(U, generator=g) * 1e-2
    dense = torch.zeros(V, K)
    dense[touched.long()] = gr
    dense_l = torch.zeros(V, 1)
    dense_l[touched.long(), 0] = gl
    E, w = E0.clone().to(cuda), w0.clone().to(cuda).reshape(-1)
    mE, vE = torch.zeros_like(E), torch.zeros_like(E)
    mw, vw = torch.zeros_like(w), torch.zeros_like(w)
    rowmap = torch.full((V,), -1, dtype=torch.int32, device=cuda)
    rowmap[touched.long().to(cuda)] = torch.arange(U, dtype=torch.int32, device=cuda)
    H.adam_embedding(E, mE, vE, w, mw, vw, rowmap, gr.to(cuda), gl.to(cuda), 1, 1e-3,
                     weight_decay=1e-5)
    assert (rowmap.cpu() == -1).all(), "rowmap must be reset by the Adam pass"
    Er, _, _ = _torch_adam_ref(E0, [dense], 1e-3, 1e-5, 1)
    wr, _, _ = _torch_adam_ref(w0, [dense_l], 1e-3, 1e-5, 1)
    np.testing.assert_allclose(E.cpu().numpy(), Er.numpy(), rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(w.cpu().numpy(), wr.numpy().reshape(-1), rtol=1e-6, atol=1e-9)
    assert not torch.equal(E.cpu()[0], E0[0]) or 0 in touched  # untouched rows moved


# --------------------------------------------------------------- Feature_Embedding ---
def test_feature_embedding_vs_golden(cuda, golden):
    H = _hip()
    g = golden("g_fe.npz")
    out = H.feature_embedding(torch.tensor(g["x"], device=cuda), torch.tensor(g["E"], device=cuda))
    # pair dots of N(0,1) rows: absolute error scales with sqrt(K)*|e|^2
    np.testing.assert_allclose(out.cpu().numpy(), g["out"], rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize("F,K", [(2, 1), (26, 64), (22, 128), (5, 3)])
def test_feature_embedding_vs_oracle(cuda, F, K):
    H = _hip()
    g = torch.Generator().manual_seed(F * K)
    V, B = 300, 45
    E = torch.randn(V, K, generator=g)
    x = torch.randint(0, V, (B, F), generator=g)
    out = H.feature_embedding(x.to(cuda), E.to(cuda)).cpu()
    ref = O.feature_embedding(E.double(), x).float()
    np.testing.assert_allclose(out.numpy(), ref.numpy(), rtol=1e-5, atol=1e-5 * K)


# ------------------------------------------------------------------- IPNN (§8f) ------
@pytest.mark.parametrize("F,K,B", [(2, 1, 3), (8, 16, 64), (26, 64, 300), (22, 128, 50),
                                   (5, 3, 7), (39, 10, 100)])
def test_ipnn_forward_and_backward_vs_oracle(cuda, F, K, B):
    """cat = flat(E[x]) ++ pair dots (p_model.py:187-195) and the per-slot gradient
    through it, against the oracle's torch-CPU ops (autograd for the backward). Flat part
    bit-exact; dots and gradients within 1e-5 of their L1 scale (sum of |terms|)."""
    H = _hip()
    g = torch.Generator().manual_seed(F * K + B)
    V = 300
    E = torch.randn(V, K, generator=g)
    x = torch.randint(0, V, (B, F), generator=g)
    x[:, 0] = x[:, 1 % F]  # a repeated id inside an example
    cat = H.ipnn_forward(x.to(cuda), E.to(cuda)).cpu()
    ref = O.ipnn_cat(E.double(), x)
    np.testing.assert_array_equal(cat[:, :F * K].numpy(), ref[:, :F * K].float().numpy())
    scale = O.ipnn_cat(E.double().abs(), x)
    assert ((cat.double() - ref).abs() <= 1e-5 * scale + 1e-30).all()
    dcat = torch.randn(B, F * K + F * (F - 1) // 2, generator=g)
    e = torch.nn.functional.embedding(x, E.double()).requires_grad_(True)
    row, col = O.ipnn_pairs(F)
    out = torch.cat([e.reshape(B, -1), (e[:, row] * e[:, col]).sum(2)], 1)
    out.backward(dcat.double())
    ds = H.ipnn_backward(x.to(cuda), E.to(cuda), dcat.to(cuda)).cpu().double().view(B, F, K)
    ea = e.detach().abs()
    pa = dcat.double().abs()[:, F * K:]
    bound = dcat.double().abs()[:, :F * K].reshape(B, F, K).clone()
    for p_, (i, j) in enumerate(zip(row.tolist(), col.tolist())):
        bound[:, i] += pa[:, p_:p_ + 1] * ea[:, j]
        bound[:, j] += pa[:, p_:p_ + 1] * ea[:, i]
    assert ((ds - e.grad).abs() <= 1e-5 * bound + 1e-30).all()


@pytest.mark.parametrize("F,K,B", [(2, 1, 3), (8, 16, 64), (26, 64, 300), (5, 3, 7),
                                   (32, 64, 33), (33, 8, 9), (22, 128, 50), (26, 16, 77),
                                   (22, 64, 41), (8, 32, 5)])
def test_ipnn_planes_and_register_backward_bitwise(cuda, F, K, B, monkeypatch):
    """ipnn_forward writing the MLP input's planes directly == split_planes of the fp32
    forward, bit for bit (with and without the fp32 copy); the register backward (F <= 32,
    K <= 64; CTR_IPNN_BWD=reg) and the scalar-operand walk (sreg, F = 26 / 22) == the
    LDS-tile backward (CTR_IPNN_BWD=lds), bit for bit; the default (the matrix-core product
    where F <= 32 and K % 32 == 0) == it within fp32 rounding, bitwise elsewhere."""
    H = _hip()
    g = torch.Generator().manual_seed(F + 7 * K + B)
    V = 500
    E = torch.randn(V, K, generator=g).to(cuda)
    x = torch.randint(0, V, (B, F), generator=g).to(cuda)
    W = F * K + F * (F - 1) // 2
    cat = H.ipnn_forward(x, E)
    want = H.split_planes(cat)
    for keep in (False, True):
        pl = H.Planes(B, W, cuda)
        out = torch.empty_like(cat) if keep else None
        H.ipnn_forward(x, E, out=out, planes=pl)
        assert torch.equal(pl.t, want.t)
        if keep:
            assert torch.equal(out, cat)
    dcat = torch.randn(B, W, generator=g).to(cuda)
    dflt = H.ipnn_backward(x, E, dcat)
    got = {}
    for mode in ("reg", "sreg", "lds"):  # sreg: the scalar-operand walk for F = 26 / 22
        monkeypatch.setenv("CTR_IPNN_BWD", mode)
        got[mode] = H.ipnn_backward(x, E, dcat)
    assert torch.equal(got["reg"], got["lds"])
    assert torch.equal(got["sreg"], got["lds"])
    lds = got["lds"]
    if F <= 32 and K % 32 == 0:
        # the matrix-core product (the default here; CTR_IPNN_BWD=m) sums in the matrix
        # core's order: within fp32 rounding of the walks (1e-5 of the largest gradient)
        torch.testing.assert_close(dflt, lds, rtol=1e-5, atol=1e-5 * float(lds.abs().max()))
        monkeypatch.setenv("CTR_IPNN_BWD", "m")
        assert torch.equal(H.ipnn_backward(x, E, dcat), dflt)  # the same on every launch
    else:
        assert torch.equal(dflt, lds)


# ------------------------------------------------------------------------ REINFORCE ---
def test_pg_discount_norm_vs_golden(cuda, golden):
    H = _hip()
    g = golden("g_pg.npz")
    r = torch.tensor(g["dn_r"], device=cuda)
    for gamma in (1.0, 0.9):
        d64, d32, stats = H.pg_discount_norm(r, gamma)
        np.testing.assert_allclose(d64.cpu().numpy(), g[f"dn_gamma{gamma}"].reshape(-1),
                                   rtol=1e-12, atol=1e-12)


def test_pg_loss_grad_vs_golden(cuda, golden):
    H = _hip()
    g = golden("g_pg.npz")
    probs = torch.softmax(torch.tensor(g["lf_logits"]), dim=1).to(cuda)
    loss, dlogits = H.pg_loss_grad(probs, torch.tensor(g["lf_acts"], device=cuda),
                                   torch.tensor(g["lf_vt"], device=cuda))
    assert loss.item() == pytest.approx(float(g["lf_loss"]), rel=1e-5)
    np.testing.assert_allclose(dlogits.cpu().numpy(), g["lf_dlogits"], rtol=1e-5, atol=1e-7)


def test_softmax_rows(cuda):
    H = _hip()
    x = torch.randn(1000, 5) * 3
    np.testing.assert_allclose(H.softmax_rows(x.to(cuda)).cpu().numpy(),
                               torch.softmax(x, 1).numpy(), rtol=1e-5, atol=1e-7)


# ------------------------------------------------------ RL ensemble (§8f rank 3) -----
@pytest.mark.parametrize("case", range(4))
def test_ensemble_preds_vs_golden(cuda, golden, case):
    """The kernel against the reference's own generate_preds outputs: rewards and
    return_c_actions bit-exact, y within 1e-6 relative (softmax / sum roundings)."""
    H = _hip()
    g = golden("g_ensemble.npz")
    k = lambda n: torch.tensor(g[f"c{case}_{n}"], device=cuda)  # noqa: E731
    y, r, rc = H.ensemble_preds(k("preds"), k("actions"), k("pw"), k("ca"), k("labels"))
    np.testing.assert_allclose(y.cpu().numpy(), g[f"c{case}_y"], rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(r.cpu().numpy(), g[f"c{case}_r"])
    np.testing.assert_array_equal(rc.cpu().numpy(), g[f"c{case}_rc"])


@pytest.mark.parametrize("B,M,dt", [(100_000, 5, torch.int64), (3000, 32, torch.int32),
                                    (1, 2, torch.int64), (2049, 7, torch.int32)])
def test_ensemble_preds_vs_oracle(cuda, B, M, dt):
    """Large and edge batches (more than one 1024-example rank chunk, M = 32, actions out of
    range, labels other than 0/1) against the oracle's per-example restatement."""
    H = _hip()
    g = torch.Generator().manual_seed(B + M)
    preds = torch.rand(B, M, generator=g)
    actions = torch.randint(0, M + 2, (B, 1), generator=g).to(dt)  # 0 and M+1: out of range
    pw = torch.softmax(torch.randn(B, M, generator=g), dim=1)
    ca = torch.rand(B, M, generator=g) * 2 - 1
    labels = torch.randint(0, 3, (B, 1), generator=g).to(dt)      # 2: neither branch
    y, r, rc = H.ensemble_preds(preds.to(cuda), actions.to(cuda), pw.to(cuda), ca.to(cuda),
                                labels.to(cuda))
    yo, ro, rco = O.ensemble_preds(preds.numpy(), actions.numpy(), pw.numpy(), ca.numpy(),
                                   labels.numpy())
    np.testing.assert_allclose(y.cpu().numpy().ravel(), yo, rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(rc.cpu().numpy(), rco)
    rr = r.cpu().numpy().ravel()
    # a reward may differ only where y and the models' mean tie to fp32 rounding
    mean = preds.numpy().mean(axis=1)
    bad = (rr != ro) & (np.abs(yo - mean) > 1e-6)
    assert not bad.any(), int(bad.sum())


def test_generate_preds_drop_in(cuda):
    """rl_ctr_prediction_amd.ensemble.generate_preds with real models (FM on HIP)."""
    from rl_ctr_prediction_amd import FM
    from rl_ctr_prediction_amd.ensemble import generate_preds
    torch.manual_seed(0)
    V, F, K, B = 500, 6, 8, 300
    models = {i: FM(V, K).to(cuda).eval() for i in range(4)}
    x = torch.randint(0, V, (B, F), device=cuda)
    g = torch.Generator().manual_seed(1)
    actions = torch.randint(1, 5, (B, 1), generator=g).to(cuda)
    pw = torch.softmax(torch.randn(B, 4, generator=g), 1).to(cuda)
    ca = (torch.rand(B, 4, generator=g) * 2 - 1).to(cuda)
    labels = torch.randint(0, 2, (B, 1), generator=g).to(cuda)
    y, r, rc = generate_preds(models, x, actions, pw, ca, labels, cuda, mode="train")
    assert y.shape == (B, 1) and r.shape == (B, 1) and rc.shape == (B, 4)
    with torch.no_grad():
        preds = torch.cat([models[i](x) for i in range(4)], 1).cpu().numpy()
    yo, ro, rco = O.ensemble_preds(preds, actions.cpu().numpy(), pw.cpu().numpy(),
                                   ca.cpu().numpy(), labels.cpu().numpy())
    np.testing.assert_allclose(y.cpu().numpy().ravel(), yo, rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(rc.cpu().numpy(), rco)


def test_colsum_multi_is_bitwise_colsum(cuda):
    """One launch pair for several column sums: each output bitwise the single colsum."""
    H = _hip()
    g = torch.Generator().manual_seed(3)
    jobs = [(torch.randn(8192, 200, generator=g), torch.randn(8192, generator=g)),
            (torch.randn(8192, 1, generator=g), None), (torch.randn(8192, 300, generator=g), None),
            (torch.randn(77, 5, generator=g), None), (torch.randn(1, 70, generator=g), None)]
    jobs = [(X.to(cuda), None if w is None else w.to(cuda)) for X, w in jobs]
    outs = [torch.empty(X.shape[1], device=cuda) for X, _ in jobs]
    H.colsum_multi([(X, w, o) for (X, w), o in zip(jobs, outs)])
    for (X, w), o in zip(jobs, outs):
        assert torch.equal(o, H.colsum(X, row_w=w)), X.shape


@pytest.mark.parametrize("shape", [(8192, 300), (8192, 1989), (200, 1664), (4, 8), (70, 130),
                                   (1, 1), (64, 1), (3, 200), (0, 5)])
def test_transpose_bitwise(cuda, shape):
    """ctr_transpose_f32 (dH1^T / X^T for the k-contiguous dW0): a bit-exact copy, ragged
    tiles and strided source rows included."""
    H = _hip()
    g = torch.Generator().manual_seed(shape[0] + shape[1])
    X = torch.randn(*shape, generator=g).to(cuda)
    assert torch.equal(H.transpose(X), X.t().contiguous())
    if shape[0] and shape[1] > 2:  # a column slice: ld_src > cols
        assert torch.equal(H.transpose(X[:, 1:-1]), X[:, 1:-1].t().contiguous())


def test_fm_step_tail_bitwise_separate_launches(cuda):
    """ctr_fm_step_tail == tensor_sum (loss, bias grad) + adam_dense at ctr[1] + step_end,
    bitwise (the FM step's dense tail, one launch)."""
    H = _hip()
    g0 = torch.Generator().manual_seed(7)
    for B, n in ((4096, 4), (1000, 7), (65536, 1)):
        loss_elem = torch.rand(B, generator=g0).to(cuda)
        gz = (torch.randn(B, generator=g0) * 1e-3).to(cuda)
        p0 = torch.randn(n, generator=g0).to(cuda)
        m0 = (torch.randn(n, generator=g0) * 1e-3).to(cuda)
        v0 = (torch.rand(n, generator=g0) * 1e-6).to(cuda)
        g_rest = (torch.randn(n, generator=g0) * 1e-3).to(cuda)
        out = {}
        for mode in ("tail", "separate"):
            tab = H.AdamStepTable(1e-3, (0.9, 0.999), cuda)
            ctr = torch.tensor([4, 5], dtype=torch.int32, device=cuda)
            p, m, v, g = p0.clone(), m0.clone(), v0.clone(), g_rest.clone()
            loss = torch.zeros(1, device=cuda)
            if mode == "tail":
                H.fm_step_tail(loss_elem, gz, 1.0 / B, loss, g[:1], p, g, m, v, tab, 5, ctr,
                               weight_decay=1e-5)
            else:
                H.tensor_sum(gz, out=g[:1])
                H.tensor_sum(loss_elem, scale=1.0 / B, out=loss)
                H.adam_dense(p, g, m, v, 5, 1e-3, weight_decay=1e-5, step_dev=ctr[1:2], table=tab)
                H.step_end(ctr)
            out[mode] = [t.cpu() for t in (loss, g, p, m, v, ctr)]
        for a, b in zip(out["tail"], out["separate"]):
            assert torch.equal(a, b), (B, n, a, b)


@pytest.mark.parametrize("B,F,dt", [(4096, 26, torch.int64), (513, 26, torch.int32),
                                    (7, 3, torch.int32), (1, 1, torch.int64)])
def test_batch_stage_copy_bitwise(cuda, B, F, dt):
    """ctr_batch_stage_copy: ids and labels into a slot in one launch, bitwise (16-B units
    where aligned, bytes otherwise: odd sizes and offset views); labels optional; anything
    but same-dtype contiguous device tensors is refused (the caller copies with torch)."""
    from rl_ctr_prediction_amd import hip_ops
    g = torch.Generator(device=cuda).manual_seed(B)
    src = torch.randint(0, 2**31 - 1, (B + 1, F), device=cuda, generator=g).to(dt)[1:]  # offset
    ys = torch.rand(B + 3, device=cuda, generator=g)[3:]
    ids, y = torch.full((B, F), -1, dtype=dt, device=cuda), torch.full((B,), -1.0, device=cuda)
    assert hip_ops.batch_stage_copy(ids, src, y, ys)
    torch.cuda.synchronize()
    assert torch.equal(ids, src) and torch.equal(y, ys)
    ids2 = torch.zeros_like(ids)
    assert hip_ops.batch_stage_copy(ids2, src)  # ids only
    torch.cuda.synchronize()
    assert torch.equal(ids2, src)
    if B > 1 and F > 1:
        assert not hip_ops.batch_stage_copy(ids2, src.t().contiguous().t())  # not contiguous
    assert not hip_ops.batch_stage_copy(ids2, src.to(torch.float32))     # other dtype
    assert not hip_ops.batch_stage_copy(ids2, src.cpu())                 # host tensor


@pytest.mark.parametrize("N,C,n_rows,seed", [(1, 1000, 5000, 0), (2, 777, 3000, 1),
                                             (8, 1024, 1_250_001, 2), (8, 300, 301, 3),
                                             (5, 64, 9, 4), (3, 1, 4, 5), (8, 4096, 40_000, 6)])
def test_sparse_plan_runs_bit_exact(cuda, N, C, n_rows, seed):
    """ctr_sparse_plan_build_runs (an owner shard's received ids: N ascending runs of unique
    rows, each padded with the spare row n_rows - 1) == the LSD plan of the same vector, bit
    for bit — including empty runs (all padding), full runs (no padding), rows every run
    holds — and leaves its mask zero."""
    from rl_ctr_prediction_amd import hip_ops
    rng = np.random.default_rng(seed)
    spare = n_rows - 1
    hot = rng.choice(spare, size=min(spare, max(1, C // 4)), replace=False) if spare else []
    runs = []
    for j in range(N):
        n = [0, C, int(rng.integers(0, C + 1))][j % 3] if N > 2 else int(rng.integers(1, C + 1))
        n = min(n, spare)
        # half of the run from the rows every run draws from (shared), the rest at random
        r = np.unique(np.concatenate([np.asarray(hot[: n // 2], dtype=np.int64),
                                      rng.choice(spare, size=n, replace=False)]))[:n]
        runs.append(np.concatenate([r, np.full(C - len(r), spare)]).astype(np.int32))
    ids = torch.tensor(np.concatenate(runs), device=cuda)
    a = hip_ops.SparsePlanBuffers(N * C, cuda).build(ids, n_rows)
    mask = torch.zeros((n_rows + 3) // 4, dtype=torch.int32, device=cuda)
    b = hip_ops.SparsePlanBuffers(N * C, cuda).build_runs(ids, N, n_rows, mask)
    b.build_runs(ids, N, n_rows, mask)  # twice: the mask came back zero
    torch.cuda.synchronize()
    U = a.num_unique_host()
    assert b.num_unique_host() == U
    S = N * C
    for name in ("sorted_slots", "sorted_rows", "pos_seg"):
        assert torch.equal(getattr(a, name)[:S], getattr(b, name)[:S]), name
    assert torch.equal(a.unique_rows[:U], b.unique_rows[:U])
    assert torch.equal(a.seg_offsets[:U + 1], b.seg_offsets[:U + 1])
    assert int(mask.abs().sum()) == 0


@pytest.mark.parametrize("n_shards", [1, 2, 3, 8, 15, 16])
@pytest.mark.parametrize("case", ["zipf", "empty", "one", "one_shard", "boundaries"])
def test_plan_shard_counts_and_max(cuda, n_shards, case):
    """ctr_plan_shard_counts(_max): per-shard unique-row counts (the wave-parallel 64-ary
    search for <= 15 shards, the per-shard binary search above) == numpy, and max_out == their
    maximum — the run length that sizes the row-sharded exchange; ctr_shard_pack_ids' padded
    exchange layout (its own per-block run search) with the same counts and offsets."""
    from rl_ctr_prediction_amd import hip_ops
    V = 1_000_003
    shard_rows = -(-V // n_shards)
    rng = np.random.default_rng(n_shards * 7 + len(case))
    if case == "zipf":
        ids = np.minimum(rng.zipf(1.2, size=8192 * 26) - 1, V - 1)
    elif case == "empty":
        ids = np.zeros(0, dtype=np.int64)
    elif case == "one":
        ids = np.array([V - 1])
    elif case == "one_shard":
        ids = rng.integers(0, min(shard_rows, V), size=50_000)
    else:  # every shard's first and last row, and their neighbours
        b = np.arange(n_shards + 1) * shard_rows
        ids = np.concatenate([b - 1, b, b + 1])
        ids = ids[(ids >= 0) & (ids < V)]
    plan = hip_ops.SparsePlanBuffers(max(ids.size, 1), cuda).build(
        torch.tensor(ids.astype(np.int64), device=cuda).reshape(1, -1) if ids.size else
        torch.zeros(0, 1, dtype=torch.int64, device=cuda), V)
    uniq = np.unique(ids)
    want = np.bincount(uniq // shard_rows, minlength=n_shards)[:n_shards].astype(np.int64)
    got = plan.shard_counts(shard_rows, n_shards).cpu().numpy()
    assert np.array_equal(got, want), (got, want)
    # the padded exchange layout (ctr_shard_pack_ids: the same run bounds, searched per block)
    C = max(int(want.max()) + 3, 1)
    send = torch.full((n_shards * C,), -7, dtype=torch.int32, device=cuda)
    cnt = torch.zeros(n_shards, dtype=torch.int32, device=cuda)
    off = torch.zeros(n_shards, dtype=torch.int32, device=cuda)
    hip_ops.shard_pack_ids(plan, shard_rows, V, n_shards, C, send, cnt, off)
    send = send.cpu().numpy().reshape(n_shards, C)
    assert np.array_equal(cnt.cpu().numpy(), want)
    assert np.array_equal(off.cpu().numpy(), np.concatenate([[0], np.cumsum(want)[:-1]]))
    for j in range(n_shards):
        run = uniq[uniq // shard_rows == j] - j * shard_rows
        spare = max(0, min(shard_rows, V - j * shard_rows))
        assert np.array_equal(send[j, :run.size], run)
        assert (send[j, run.size:] == spare).all()
    if n_shards <= 15:
        mx = torch.full((1,), -1, dtype=torch.int64, device=cuda)
        got2 = plan.shard_counts(shard_rows, n_shards, max_out=mx).cpu().numpy()
        assert np.array_equal(got2, want)
        assert int(mx.item()) == int(want.max()), (int(mx.item()), want)
    else:
        with pytest.raises(Exception, match="15 shards"):
            plan.shard_counts(shard_rows, n_shards,
                              max_out=torch.zeros(1, dtype=torch.int64, device=cuda))


@pytest.mark.parametrize("n,C,K,lin", [(1, 1024, 64, True), (3, 1000, 16, True), (8, 37, 4, False),
                                       (2, 5, 8, True)])
def test_shard_rows_lin_exchange_layout(cuda, n, C, K, lin):
    """The chunked rows + linear-weight exchange (ctr_shard_gather_rows / _rows_pack /
    _rows_unpack) == the layout written out with numpy: chunk j = [C rows][C weights][pad];
    pack zero-fills past each run, unpack restores exactly the runs, gather reads the ids."""
    from rl_ctr_prediction_amd import hip_ops
    rng = np.random.default_rng(n * C + K)
    Vo = 500
    E = rng.standard_normal((Vo, K)).astype(np.float32)
    w = rng.standard_normal(Vo).astype(np.float32)
    counts = rng.integers(0, C + 1, size=n).astype(np.int32)
    offsets = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int32)
    U = int(counts.sum())
    chunk = hip_ops.rows_chunk(C, K, lin)
    assert chunk % 4 == 0 and chunk >= C * K + (C if lin else 0)
    d = lambda a: torch.tensor(a, device=cuda)  # noqa: E731
    # gather (owner side): chunk j row i = E[ids[j*C+i]], w[ids[j*C+i]]
    ids = rng.integers(0, Vo, size=n * C).astype(np.int32)
    out = torch.full((n * chunk,), float("nan"), device=cuda)
    hip_ops.shard_gather_rows(d(E), d(w) if lin else None, d(ids), n, C, out=out)
    o = out.cpu().numpy().reshape(n, chunk)
    for j in range(n):
        assert np.array_equal(o[j, :C * K].reshape(C, K), E[ids[j * C:(j + 1) * C]])
        if lin:
            assert np.array_equal(o[j, C * K:C * K + C], w[ids[j * C:(j + 1) * C]])
    # pack: compact rows -> chunks, zeros past each run
    rows = rng.standard_normal((max(U, 1), K)).astype(np.float32)
    lv = rng.standard_normal(max(U, 1)).astype(np.float32)
    out = torch.full((n * chunk,), float("nan"), device=cuda)
    hip_ops.shard_rows_pack(d(rows), d(lv) if lin else None, C, d(counts), d(offsets), out=out)
    o = out.cpu().numpy().reshape(n, chunk)
    for j in range(n):
        c, f = counts[j], offsets[j]
        blk = o[j, :C * K].reshape(C, K)
        assert np.array_equal(blk[:c], rows[f:f + c]) and (blk[c:] == 0).all()
        if lin:
            assert np.array_equal(o[j, C * K:C * K + c], lv[f:f + c])
            assert (o[j, C * K + c:C * K + C] == 0).all()
    # unpack: the chunks back to the runs (rows past U untouched)
    back = torch.full((max(U, 1) + 3, K), -5.0, device=cuda)
    backl = torch.full((max(U, 1) + 3,), -5.0, device=cuda)
    hip_ops.shard_rows_unpack(out, C, d(counts), d(offsets), back, backl if lin else None)
    assert np.array_equal(back.cpu().numpy()[:U], rows[:U])
    assert (back.cpu().numpy()[max(U, 1):] == -5.0).all()
    if lin:
        assert np.array_equal(backl.cpu().numpy()[:U], lv[:U])


@pytest.mark.parametrize("K,lin", [(64, True), (16, True), (32, False)])
def test_adam_deferred_entries_equals_sums_then_rows(cuda, K, lin):
    """ctr_adam_deferred_entries (the row-sharded owner: each row's entries summed straight,
    then replayed + stepped) == numpy's sequential fp32 sums in plan order, and the table after
    it == ctr_adam_deferred_rows with grad_rows = those sums, bitwise; the same read from the
    chunked exchange layout (run_len = C); skip_row untouched."""
    from rl_ctr_prediction_amd import hip_ops as H
    rng = np.random.default_rng(K)
    Vo, n, C = 3000, 4, 700
    spare = Vo - 1
    # n runs of ascending unique rows padded with the spare row: each row <= n entries
    ids = np.full((n, C), spare, dtype=np.int32)
    for j in range(n):
        cnt = rng.integers(C // 2, C)
        ids[j, :cnt] = np.sort(rng.choice(spare, size=cnt, replace=False))
    ids = ids.reshape(-1)
    vals = rng.standard_normal((n * C, K)).astype(np.float32) * 1e-2
    vlin = rng.standard_normal(n * C).astype(np.float32) * 1e-2
    d = lambda a: torch.tensor(a, device=cuda)  # noqa: E731
    plan = H.SparsePlanBuffers(n * C, cuda).build(d(ids), Vo)
    tab = H.AdamStepTable(1e-3, (0.9, 0.999), cuda)
    E0 = rng.standard_normal((Vo, K)).astype(np.float32) * 0.05
    w0 = rng.standard_normal(Vo).astype(np.float32) * 0.05
    last0 = rng.integers(0, 6, size=Vo).astype(np.int32)  # rows 0..5 steps behind
    step = 7

    def state():
        z = lambda *s: torch.zeros(*s, device=cuda)  # noqa: E731
        st = [d(E0), z(Vo, K), z(Vo, K)]
        st += [d(w0), z(Vo), z(Vo)] if lin else [None, None, None]
        return st + [d(last0)]

    a = state()
    U = plan.num_unique_host()
    sums = torch.zeros(n * C, K, device=cuda)
    slin = torch.zeros(n * C, device=cuda)
    H.adam_deferred_entries(*a, plan, d(vals), d(vlin) if lin else None, step, tab,
                            weight_decay=1e-5, skip_row=spare, out=sums,
                            out_lin=slin if lin else None)
    # numpy: sequential sums in plan order
    srt = plan.sorted_slots[:n * C].cpu().numpy()
    offs = plan.seg_offsets[:U + 1].cpu().numpy()
    urows = plan.unique_rows[:U].cpu().numpy()
    want = np.zeros((U, K), np.float32)
    want_l = np.zeros(U, np.float32)
    for u in range(U):
        if urows[u] == spare:
            continue
        e = srt[offs[u]:offs[u + 1]]
        acc, accl = vals[e[0]].copy(), np.float32(vlin[e[0]])
        for x in e[1:]:
            acc = (acc + vals[x]).astype(np.float32)
            accl = np.float32(accl + vlin[x])
        want[u], want_l[u] = acc, accl
    # the same from the exchange's chunked receive buffer (run_len = C): bitwise
    chunk = H.rows_chunk(C, K, lin)
    buf = np.zeros((n, chunk), np.float32)
    for j in range(n):
        buf[j, :C * K] = vals[j * C:(j + 1) * C].reshape(-1)
        if lin:
            buf[j, C * K:C * K + C] = vlin[j * C:(j + 1) * C]
    cst = state()
    H.adam_deferred_entries(*cst, plan, d(buf.reshape(-1)), None, step, tab, weight_decay=1e-5,
                            skip_row=spare, run_len=C)
    for x, y in zip(a, cst):
        if x is not None:
            assert torch.equal(x, y)
    live = urows != spare
    got = sums[:U].cpu().numpy()
    assert np.array_equal(got[live], want[live])
    if lin:
        assert np.array_equal(slin[:U].cpu().numpy()[live], want_l[live])
    # the same update from the sums through ctr_adam_deferred_rows
    b = state()
    grows = torch.tensor(np.where(live[:, None], want, 0), device=cuda)
    glin = torch.tensor(np.where(live, want_l, 0), device=cuda) if lin else None
    H.adam_deferred_rows(*b, plan, step, tab, weight_decay=1e-5, grad_rows=grows,
                         grad_lin=glin)
    rows_live = torch.tensor(urows[live].astype(np.int64), device=cuda)
    for x, y in zip(a, b):
        if x is None:
            continue
        assert torch.equal(x[rows_live], y[rows_live])
    assert torch.equal(a[0][spare], d(E0)[spare]) and int(a[-1][spare]) == last0[spare]


@pytest.mark.parametrize("mode", ["fm", "vals"])
def test_shard_row_grads_into_chunks(cuda, mode):
    """ctr_shard_row_grads == the compact per-row sums (ctr_fm_embedding_grad compact /
    ctr_segment_sum_rows) then ctr_shard_rows_pack, bitwise on every run row and linear sum."""
    from rl_ctr_prediction_amd import hip_ops as H
    rng = np.random.default_rng(3 if mode == "fm" else 4)
    B, F, K, V = 512, 6, 16, 5000
    x = torch.tensor(rng.integers(0, V, size=(B, F)), device=cuda)
    plan = H.SparsePlanBuffers(B * F, cuda).build(x, V)
    U = plan.num_unique_host()
    n = 3
    cuts = np.sort(rng.choice(np.arange(1, U), size=n - 1, replace=False))
    counts = np.diff(np.concatenate([[0], cuts, [U]])).astype(np.int32)
    offsets = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int32)
    C = int(counts.max()) + 5
    d = lambda a: torch.tensor(a, device=cuda)  # noqa: E731
    lin = mode == "fm"
    chunk = H.rows_chunk(C, K, lin)
    got = torch.zeros(n * chunk, device=cuda)
    if mode == "fm":
        T = d(rng.standard_normal((U, K)).astype(np.float32))
        gz = d(rng.standard_normal(B).astype(np.float32))
        sum_e = d(rng.standard_normal((B, K)).astype(np.float32))
        dx = d(rng.standard_normal((B, F * K)).astype(np.float32))
        gr, gl = H.fm_embedding_grad(plan, F, T, gz, sum_e, dx, compact=True)
        H.shard_row_grads(plan, C, d(offsets), got, K=K, F=F, emb=T, gz=gz, sum_e=sum_e, dx=dx,
                          lin=True)
    else:
        vals = d(rng.standard_normal((B * F, K)).astype(np.float32))
        gr, gl = H.segment_sum_rows(plan, vals)
        H.shard_row_grads(plan, C, d(offsets), got, K=K, vals=vals)
    want = torch.zeros(n * chunk, device=cuda)
    H.shard_rows_pack(gr[:max(U, 1)].contiguous(), gl[:max(U, 1)].contiguous() if lin else None,
                      C, d(counts), d(offsets), out=want)
    g, w = got.view(n, chunk), want.view(n, chunk)
    for j in range(n):
        c = int(counts[j])
        assert torch.equal(g[j, :c * K], w[j, :c * K]), j
        if lin:
            assert torch.equal(g[j, C * K:C * K + c], w[j, C * K:C * K + c]), j


@pytest.mark.parametrize("mode", ["fm", "vals"])
def test_shard_row_grads_capacity_overflow_stays_in_chunk(cuda, mode):
    """A run longer than the capacity C (the case shard_pack_ids flags with
    CTR_EFLAG_CAPACITY) writes its first C rows and nothing past its own chunk: every row and
    linear slot beyond min(count, C) keeps its sentinel, and the first min(count, C) rows are
    the pack kernel's (which clamps the same way)."""
    from rl_ctr_prediction_amd import hip_ops as H
    rng = np.random.default_rng(11 if mode == "fm" else 12)
    B, F, K, V = 256, 6, 16, 3000
    x = torch.tensor(rng.integers(0, V, size=(B, F)), device=cuda)
    plan = H.SparsePlanBuffers(B * F, cuda).build(x, V)
    U = plan.num_unique_host()
    n = 3
    counts = np.array([U // 2, U // 4, U - U // 2 - U // 4], np.int32)
    offsets = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int32)
    C = int(counts[1]) + 3  # run 0 (and maybe run 2) overflow
    assert counts.max() > C
    d = lambda a: torch.tensor(a, device=cuda)  # noqa: E731
    lin = mode == "fm"
    chunk = H.rows_chunk(C, K, lin)
    sentinel = 12345.0
    got = torch.full((n * chunk,), sentinel, device=cuda)
    if mode == "fm":
        T = d(rng.standard_normal((U, K)).astype(np.float32))
        gz = d(rng.standard_normal(B).astype(np.float32))
        sum_e = d(rng.standard_normal((B, K)).astype(np.float32))
        dx = d(rng.standard_normal((B, F * K)).astype(np.float32))
        gr, gl = H.fm_embedding_grad(plan, F, T, gz, sum_e, dx, compact=True)
        H.shard_row_grads(plan, C, d(offsets), got, K=K, F=F, emb=T, gz=gz, sum_e=sum_e, dx=dx,
                          lin=True)
    else:
        vals = d(rng.standard_normal((B * F, K)).astype(np.float32))
        gr, gl = H.segment_sum_rows(plan, vals)
        H.shard_row_grads(plan, C, d(offsets), got, K=K, vals=vals)
    torch.cuda.synchronize()
    want = torch.zeros(n * chunk, device=cuda)
    H.shard_rows_pack(gr[:U].contiguous(), gl[:U].contiguous() if lin else None, C, d(counts),
                      d(offsets), out=want)
    g, w = got.view(n, chunk), want.view(n, chunk)
    for j in range(n):
        m = min(int(counts[j]), C)
        assert torch.equal(g[j, :m * K], w[j, :m * K]), j
        assert bool((g[j, m * K:C * K] == sentinel).all()), j
        if lin:
            assert torch.equal(g[j, C * K:C * K + m], w[j, C * K:C * K + m]), j
            assert bool((g[j, C * K + m:] == sentinel).all()), j
        else:
            assert bool((g[j, C * K:] == sentinel).all()), j


@pytest.mark.parametrize("dtype", [torch.int64, torch.int32])
def test_shard_permute_ids_and_cyclic_pack(cuda, dtype):
    """Cyclic row sharding: ctr_shard_permute_ids maps r -> (r % N) * Vs + r // N in place
    (bit-exact vs numpy; ids outside [0, V) raise CTR_EFLAG_INDEX and map to row 0), the plan
    over the permuted ids groups its unique rows by owner, and ctr_shard_pack_ids_layout
    packs each owner's run as owner-local ids r // N padded with the owner's cyclic row count
    ceil((V - j) / N) (its spare row)."""
    from rl_ctr_prediction_amd import hip_ops as H
    rng = np.random.default_rng(5)
    V, N, B, F = 10_007, 4, 300, 7
    Vs = -(-V // N)
    x = rng.integers(0, V, size=(B, F))
    got = torch.tensor(x, dtype=dtype, device=cuda)
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    H.shard_permute_ids_(got, V, N, Vs, err_flag=err)
    want = (x % N) * Vs + x // N
    assert np.array_equal(got.cpu().numpy(), want) and int(err) == 0
    bad = torch.tensor([[0, V, -1, V - 1]], dtype=dtype, device=cuda)
    H.shard_permute_ids_(bad, V, N, Vs, err_flag=err)
    assert int(err) != 0
    assert bad.cpu().tolist() == [[0, 0, 0, ((V - 1) % N) * Vs + (V - 1) // N]]
    plan = H.SparsePlanBuffers(B * F, cuda).build(got, N * Vs)
    U = plan.num_unique_host()
    urows = plan.unique_rows[:U].cpu().numpy()
    assert np.array_equal(urows, np.unique(want))
    C = 512
    send = torch.empty(N * C, dtype=torch.int32, device=cuda)
    counts = torch.empty(N, dtype=torch.int32, device=cuda)
    offsets = torch.empty(N, dtype=torch.int32, device=cuda)
    H.shard_pack_ids(plan, Vs, V, N, C, send, counts, offsets, cyclic=True)
    s = send.view(N, C).cpu().numpy()
    orig = np.unique(x)
    for j in range(N):
        mine = orig[orig % N == j] // N
        assert int(counts[j]) == len(mine)
        assert np.array_equal(s[j, :len(mine)], mine), j
        assert (s[j, len(mine):] == len(range(j, V, N))).all(), j


def test_cu_masked_stream_runs_kernels(cuda):
    """ctr_stream_create_cu_masked: a stream on half the CUs (hip_ops.cu_masked_stream) runs
    the library's kernels with the same results as the default stream (the permute kernel,
    bit-exact), and ctr_stream_destroy releases a stream it made."""
    from rl_ctr_prediction_amd import hip_ops as H
    from rl_ctr_prediction_amd._lib import lib
    n_cus = torch.cuda.get_device_properties(cuda).multi_processor_count
    st = H.cu_masked_stream(H.cu_mask_words(n_cus, 0.5), device=cuda)
    V, N = 1000, 3
    Vs = -(-V // N)
    ids = torch.randint(0, V, (4096,), device=cuda, generator=torch.Generator(cuda).manual_seed(5))
    ref = H.shard_permute_ids_(ids.clone(), V, N, Vs)
    torch.cuda.synchronize()
    with torch.cuda.stream(st):
        got = H.shard_permute_ids_(ids.clone(), V, N, Vs)
    st.synchronize()
    assert torch.equal(got, ref)
    import ctypes
    h = ctypes.c_void_p()
    words = (ctypes.c_uint32 * 1)(0xFFFF)
    lib.ctr_stream_create_cu_masked(ctypes.addressof(words), 1, ctypes.addressof(h))
    assert h.value
    lib.ctr_stream_destroy(h.value)
