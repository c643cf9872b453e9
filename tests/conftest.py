"""Shared pytest setup: repo root on sys.path, the `gpu` marker, golden loaders."""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm device) and libctr_hip.so")


def load_golden(name: str):
    p = GOLDEN / name
    if p.suffix == ".json":
        return json.loads(p.read_text())
    return np.load(p, allow_pickle=False)


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no ROCm device is visible")
    from rl_ctr_prediction_amd._lib import lib
    lib.load()  # the HIP library must load: no fallback
    return torch.device("cuda:0")


class AdamBound:
    """Per-element interval of Adam-updated parameters (torch.optim.Adam, the reference's
    optimizer, all_main/pretrain_main.py:153): the parity bar for parameters after Adam.

    Adam's step lr*m^/(sqrt(v^)+eps) is scale-invariant in the gradient and steep where
    |g| ~ eps: there a 1e-9 gradient difference moves the step by a few % of lr, so a
    fixed rtol cannot hold on every element while a loose one hides real errors. Instead
    the recurrences are evaluated in interval arithmetic (float64): given each step's
    reference gradient g and the per-element gradient bound `gtol` that the test checked
    (|ours - g| <= gtol, from assert_grad_close), the parameter, m and v intervals contain
    every value Adam can produce from any gradient within the bound; weight decay uses the
    parameter interval. check() then asserts EVERY element inside its interval widened by
    fp32 rounding (a few ulp of the parameter and of the step per step) — no fraction
    of elements is exempt. The reference's own values must lie inside too (checks the
    bound model)."""

    def __init__(self, p0, lr, weight_decay, betas=(0.9, 0.999), eps=1e-8):
        p0 = np.asarray(p0, dtype=np.float64)
        self.lo, self.hi = p0.copy(), p0.copy()
        self.lr, self.wd, (self.b1, self.b2), self.eps = lr, weight_decay, betas, eps
        self.slack = np.zeros_like(p0)
        self.reset()

    def reset(self):
        """A fresh torch.optim.Adam (the reference re-creates it every epoch)."""
        self.m_lo = np.zeros_like(self.lo)
        self.m_hi = np.zeros_like(self.lo)
        self.v_lo = np.zeros_like(self.lo)
        self.v_hi = np.zeros_like(self.lo)
        self.t = 0

    def step(self, g, gtol, lr=None):
        lr = self.lr if lr is None else lr
        b1, b2 = self.b1, self.b2
        g = np.asarray(g, dtype=np.float64).reshape(self.lo.shape)
        gtol = np.broadcast_to(np.asarray(gtol, dtype=np.float64), self.lo.shape)
        self.t += 1
        glo = g - gtol + self.wd * self.lo
        ghi = g + gtol + self.wd * self.hi
        self.m_lo = b1 * self.m_lo + (1 - b1) * glo
        self.m_hi = b1 * self.m_hi + (1 - b1) * ghi
        sq_lo = np.where((glo <= 0) & (ghi >= 0), 0.0, np.minimum(glo * glo, ghi * ghi))
        sq_hi = np.maximum(glo * glo, ghi * ghi)
        self.v_lo = b2 * self.v_lo + (1 - b2) * sq_lo
        self.v_hi = b2 * self.v_hi + (1 - b2) * sq_hi
        bc1, bc2 = 1 - b1 ** self.t, 1 - b2 ** self.t
        n_lo, n_hi = lr * self.m_lo / bc1, lr * self.m_hi / bc1
        d_lo = np.sqrt(self.v_lo / bc2) + self.eps
        d_hi = np.sqrt(self.v_hi / bc2) + self.eps
        u_lo = np.where(n_lo >= 0, n_lo / d_hi, n_lo / d_lo)
        u_hi = np.where(n_hi >= 0, n_hi / d_lo, n_hi / d_hi)
        self.lo, self.hi = self.lo - u_hi, self.hi - u_lo
        # fp32 rounding of both implementations: the parameter store and the step's ~6
        # dependent roundings (m, v, sqrt, +eps, divide, multiply), generously
        umax = np.maximum(np.abs(u_lo), np.abs(u_hi))
        self.slack += 2.0 ** -22 * np.maximum(np.abs(self.lo), np.abs(self.hi)) + 2.0 ** -20 * umax
        return self

    def check(self, actual, desired=None, err_msg=""):
        a = np.asarray(actual, dtype=np.float64).reshape(self.lo.shape)
        lo, hi = self.lo - self.slack - 1e-30, self.hi + self.slack + 1e-30
        for name, v in (("actual", a), ("reference", desired)):
            if v is None:
                continue
            v = np.asarray(v, dtype=np.float64).reshape(self.lo.shape)
            bad = (v < lo) | (v > hi)
            if bad.any():
                i = np.flatnonzero(bad.reshape(-1))[0]
                raise AssertionError(
                    f"{err_msg}: {int(bad.sum())}/{bad.size} {name} elements outside the Adam "
                    f"interval; first at flat {i}: {v.reshape(-1)[i]!r} not in "
                    f"[{lo.reshape(-1)[i]!r}, {hi.reshape(-1)[i]!r}]")

    def take(self, idx):
        """The bound restricted to rows idx (sampled comparisons of large tables)."""
        out = AdamBound.__new__(AdamBound)
        out.__dict__.update({k: (v[idx] if isinstance(v, np.ndarray) else v)
                             for k, v in self.__dict__.items()})
        return out


def assert_grad_close(actual, desired, *, rtol=1e-5, atol_frac=1e-6, cond=None, n_terms=None,
                      err_msg=""):
    """Gradients: 1e-5 relative, with an absolute floor of 1e-6 x the tensor's largest
    magnitude, or — when `cond` (the per-element L1 norm of the summands,
    oracle.grad_condition) is given — 1e-5 x cond: a row gradient is a sum over up to ~1e4
    slot terms and, under cancellation, only its error relative to the terms is meaningful.

    `n_terms` (slots summed into each row): fp32 summation of n terms in two different
    association orders (the reference's sequential chain vs the chunked deterministic sum)
    differs by ~u*sqrt(n)*cond per implementation (u = 2^-24, random-walk rounding); the
    bound used is max(rtol, 8*u*sqrt(n)) x cond, which equals the 1e-5 bar for rows of up to
    ~430 slots and only widens for the hot Zipf rows (n ~ 8k: 4.9e-5).

    Returns the per-element bound it checked (the gradient error AdamBound.step propagates)."""
    a = np.asarray(actual, dtype=np.float64)
    d = np.asarray(desired, dtype=np.float64)
    tol = grad_bound(d, rtol=rtol, atol_frac=atol_frac, cond=cond, n_terms=n_terms)
    bad = np.abs(a - d) > tol
    if bad.any():
        i = np.flatnonzero(bad.reshape(-1))[0]
        raise AssertionError(
            f"{err_msg}: {int(bad.sum())}/{bad.size} gradient elements outside the bar "
            f"({'1e-5*|g| + max(1e-5, 8u*sqrt(n))*sum|terms|' if cond is not None else '1e-5*|g| + 1e-6*max|g|'}); "
            f"first at flat {i}: {a.reshape(-1)[i]!r} vs {d.reshape(-1)[i]!r}, "
            f"max excess {np.max(np.abs(a - d) - tol):.3g}")
    return tol


def grad_bound(desired, *, rtol=1e-5, atol_frac=1e-6, cond=None, n_terms=None):
    """The per-element gradient bar of assert_grad_close (see there)."""
    d = np.asarray(desired, dtype=np.float64)
    if cond is None:
        return rtol * np.abs(d) + atol_frac * max(np.abs(d).max(), 1e-30)
    c = np.asarray(cond, dtype=np.float64)
    crel = np.full(c.shape, rtol)
    if n_terms is not None:
        n = np.asarray(n_terms, dtype=np.float64).reshape((-1,) + (1,) * (c.ndim - 1))
        crel = np.maximum(crel, 8.0 * 2.0 ** -24 * np.sqrt(n))
    return rtol * np.abs(d) + crel * c + 1e-30


def fused_grads(tr):
    """A FusedCTRTrainer's last-step gradients, densified on the host:
    (E grad [V,K], w grad [V,1] or None, {dense name: grad})."""
    import torch
    assert getattr(tr, "keep_grads", True), "set tr.keep_grads = True before stepping"
    tr._drain_tail()  # a pipelined trainer's last dW0 (and its MLP Adam) is still pending
    b = tr._bufs
    U = b.plan.num_unique_host()
    rows = b.plan.unique_rows[:U].long()
    gE = torch.zeros(tr.V, tr.K, device=tr.device)
    gE[rows] = b.grad_rows[:U]
    gw = None
    if tr.w_tab is not None:
        gw = torch.zeros(tr.V, 1, device=tr.device)
        gw[rows, 0] = b.grad_lin[:U]
        gw = gw.cpu().numpy()
    dense = {n: v.detach().cpu().numpy() for n, v in tr.grad_views.items()}
    return gE.cpu().numpy(), gw, dense


def pred_deviation(actual, desired) -> float:
    """Largest deviation of predicted probabilities in logit space, relative to the logit:
    max |logit(a) - logit(d)| / (|logit(d)| + 1) over the predictions strictly inside (0, 1)
    in both; predictions at exactly 0 or 1 (fp32 sigmoid saturation) must match within 1e-6
    absolute, and otherwise count as an infinite deviation. A sigmoid output's relative error
    is (1 - p) times its logit's absolute error, so comparing p relatively punishes
    saturated predictions (p ~ 1e-30 with logits ~ -70) for last-bit logit differences."""
    a = np.asarray(actual, dtype=np.float64).reshape(-1)
    d = np.asarray(desired, dtype=np.float64).reshape(-1)
    inside = (a > 0) & (a < 1) & (d > 0) & (d < 1)
    if (np.abs(a - d)[~inside] > 1e-6).any():
        return float("inf")
    if not inside.any():
        return 0.0
    za = np.log(a[inside]) - np.log1p(-a[inside])
    zd = np.log(d[inside]) - np.log1p(-d[inside])
    return float(np.max(np.abs(za - zd) / (np.abs(zd) + 1.0)))


def assert_preds_within_spread(actual, desired, spread_key, *, factor=2.0, err_msg=""):
    """Multi-epoch driver predictions vs the reference's run. The bar is the larger of the
    1e-5 north-star tolerance and `factor` x the spread of the reference's own fp32 arithmetic
    (toy_spread.json, make_toy_spread.py: the oracle at 1/2/3/4/8 CPU threads, with the
    transposed GEMM, and with the FM sums in reverse order — equally valid evaluation orders
    of the reference's formulas — deviates from the recorded run by up to 1.7e-5 (FM) and
    1.3e-4 (DeepFM, day split) after five epochs of training, which amplify last-bit
    differences), both in pred_deviation's logit space."""
    kind, run = spread_key
    spread = load_golden("toy_spread.json")[kind][run]["max"]
    bar = max(1e-5, factor * spread)
    dev = pred_deviation(actual, desired)
    assert dev <= bar, (f"{err_msg}: prediction deviation {dev:.3g} > bar {bar:.3g} "
                        f"(reference spread {spread:.3g})")
    return dev


def collect_ranks(procs, q, n, timeout=240.0):
    """n results from the rank processes' queue; fails at once when a rank exits with an
    error (its peers would otherwise wait in a collective until the timeout), and prints
    a heartbeat so a long multi-process test is not mistaken for a hung one."""
    import queue
    import sys
    import time
    out, t0, beat = [], time.time(), time.time()
    while len(out) < n:
        try:
            out.append(q.get(timeout=5))
            continue
        except queue.Empty:
            pass
        dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
        if dead:
            for p in procs:
                if p.is_alive():
                    p.kill()
            raise AssertionError(f"a rank process failed (exit codes {dead})")
        if time.time() - t0 > timeout:
            for p in procs:
                if p.is_alive():
                    p.kill()
            raise AssertionError(f"ranks timed out after {timeout:.0f} s")
        if time.time() - beat > 30:
            print(f"[ranks] waiting {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
            beat = time.time()
    return out
