"""Benchmark: CTR training examples/sec of the fused HIP step (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4|c5] [--no-cpu-baseline]

N>1 is launched by the driver as `python -m torch.distributed.run --nproc-per-node N ...`:
one process per GPU, RCCL over xGMI, data parallel with row-sharded embedding tables
(ShardedCTRTrainer: ids / rows / row gradients by all-to-all, dense gradients all-reduced;
--sharding replicated keeps full replicas with a sparse all-gather: a comparison mode, eager,
one host read per step — DESIGN.md §6). Weak scaling: every
rank trains its own B-example batches; value = all ranks' examples / max time.

Workload (default c3 = BASELINE configs[2], the north-star target shape): DeepFM, 26
fields, 10M-id vocabulary, embed_dim 64, batch 8192 per GPU, synthetic Criteo-shape ids
(skewed field cardinalities, Zipf(1.1) within fields) and planted-FM labels, inputs
resident in HBM, reference semantics (dense Adam, lr 1e-3, wd 1e-5, dropout 0.2).
c2 = configs[1]: FM, 1M vocab, dim 16, batch 4096.
c4 = configs[3]: REINFORCE (PolicyGradient.learn) over Feature_Embedding states of the C2
table, policy MLP 741-1024-512-256-128-5, episode 4096 transitions per GPU; N>1 splits
one episode over the ranks with the single-process result (pg_model.py).
c5 = configs[4]: FM, Avazu-shape 22 fields, 40M vocab, dim 128, batch 8192 per GPU; N>1
row-shards the table across the ranks (all-to-all), the configuration it is quoted on.

The JSON line carries `roofline` for the dominant kernel group of the step — chosen by an
un-timed breakdown pass among the MLP GEMMs (C3/IPNN: gemm_planes_kernel, fp32-equivalent
TFLOP/s against the fp32 MFMA peak), the deferred-Adam flush (C2/C5: deferred_flush_tile,
HBM GB/s: 24 B per element + 8 B per row), the gather, the sparse plan, the scatter and the
Adam row passes — with its per-launch duration measured by HIP events on the launch stream
in eager steps right after the timed region; and `cpu_baseline` (the oracle = torch-CPU
restatement of the reference, timed on this host's cores on a bounded sample of the same
workload, rank 0 at N=1, with the CPU model named).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "CTR train examples/sec at 1/2/4/8 MI355X; HBM GB/s on embedding gather/scatter"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
MFMA_F32_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: FP32 matrix (v_mfma_f32_32x32x2_f32), spec
MFMA_BF16_PEAK_TFS = 2500.0  # MI355X_MICROARCH.md: BF16 MFMA dense (the split GEMM's pipe)

CONFIGS = {
    "c3": dict(kind="DeepFM", V=10_000_000, F=26, K=64, B=8192,
               workload="C3 DeepFM (FM + MLP 1664-300-200-1), Criteo-shape 26 fields, "
                        "10M vocab, embed_dim 64, batch 8192/GPU"),
    "c2": dict(kind="FM", V=1_000_000, F=26, K=16, B=4096,
               workload="C2 FM, Criteo-shape 26 fields, 1M vocab, embed_dim 16, batch 4096/GPU"),
    "c4": dict(kind="PG", V=1_000_000, F=26, K=16, B=4096, A=5,
               workload="C4 REINFORCE PolicyGradient.learn: Feature_Embedding state (C2 table, "
                        "325 pairs + 416) -> policy MLP 741-1024-512-256-128-5, episode "
                        "4096 transitions/GPU"),
    "c5": dict(kind="FM", V=40_000_000, F=22, K=128, B=8192,
               workload="C5 FM, Avazu-shape 22 fields, 40M vocab, embed_dim 128, batch 8192/GPU"),
    # SURVEY.md §8f rank 1 (not a BASELINE config): InnerPNN at the C3 shape
    "ipnn": dict(kind="IPNN", V=10_000_000, F=26, K=64, B=8192,
                 workload="IPNN (flat ++ 325 pair dots -> MLP 1989-300-200-1), Criteo-shape 26 "
                          "fields, 10M vocab, embed_dim 64, batch 8192/GPU"),
}
MLP_KINDS = ("DeepFM", "IPNN")


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def adam_bytes(V, K, U):
    """Algorithmic bytes of one dense-Adam pass over E[V,K] + w[V]:
    read+write p, m, v for every element (24 B), the rowmap read (4 B/row), and for the
    U rows present in the batch their gradient row (4K B), linear grad (4 B) and the
    rowmap reset (4 B)."""
    return 24 * V * (K + 1) + 4 * V + U * (4 * K + 8)


def gather_bytes(S, K, B, deep, planes=True):
    """fm_forward: int64 ids (8 B/slot), the gathered row (4K B) and linear weight (4 B)
    per slot, the per-example sums written (4K B/example), and for DeepFM the MLP input
    written — as its three bf16 planes (6K B/slot, fm_forward_planes: the default) or fp32
    (4K B/slot)."""
    x_bytes = (6 if planes else 4) * K
    return S * (8 + 4 * K + 4) + B * 4 * K + (S * x_bytes if deep else 0) + B * 16


def ipnn_gather_bytes(S, K, B, F):
    """ipnn_forward_kernel: int64 ids (8 B/slot) and the gathered row (4K B/slot) read, the MLP
    input [B, F*K + F(F-1)/2] written (fp32)."""
    return S * (8 + 4 * K) + B * 4 * (F * K + F * (F - 1) // 2)


def scatter_bytes(S, K, U, deep, apply=False):
    """fm_embedding_grad: per slot its plan entries (12 B) and example terms (4 B gz +
    4K B sum_e), for DeepFM the MLP-input gradient row (4K B); per unique row the table
    row read, the gradient row written (4K B each) and the linear grad (4 B). apply (the
    fused deferred-Adam apply of N = 1, ctr_fm_embedding_grad_adam): per unique row also
    read + write p, m, v of the row and of its linear weight (24 (K + 1) B) and last[]."""
    return (S * (12 + 4 + 4 * K + (4 * K if deep else 0)) + U * (8 * K + 8)
            + (U * (24 * (K + 1) + 8) if apply else 0))


def plan_bytes(S, U):
    """Sparse plan, algorithmic: read the ids (8 B/slot), write sorted slots, sorted rows
    and slot->segment (12 B/slot), unique rows and segment offsets (8 B/unique)."""
    return S * 20 + U * 8


def gemm_planes_bytes(M, N, K, out_planes=False, aux=False):
    """One MLP GEMM on pre-split operands, algorithmic: both operands' three bf16 planes read
    once (6 B per element), the fp32 output written (4 B), its planes too when the next GEMM
    reads them (6 B), the epilogue's fp32 aux operand read (4 B)."""
    return 6 * (M * K + K * N) + M * N * (4 + (6 if out_planes else 0) + (4 if aux else 0))


def step_model(kind, B, F, K, U, H1=300, H2=200, flush_bytes_per_step=0.0, lin=True):
    """Algorithmic HBM bytes and flops of one training step as the timed region runs it
    (N = 1, deferred-exact Adam, plan built ahead; DESIGN.md §5 "step roofline"): the plan
    (S·20 + U·8), the catch-up of the batch's U rows (U·(24(K+1) + 8): p, m, v of the row
    and of its linear weight read + written, last[] read + written), the gather + forward,
    the MLP GEMMs (planes bytes, 2·M·N·K flops), the head, the per-row sums with the fused
    Adam apply of the U rows, the dense Adam and the flush amortised over the region's
    steps. Returns {part: bytes}, flops."""
    S = B * F
    deep = kind in MLP_KINDS
    parts = {"plan": plan_bytes(S, U),
             "catchup": U * (24 * (K + (1 if lin else 0)) + 8)}
    flops = 0.0
    if kind == "IPNN":
        W = F * K + F * (F - 1) // 2
        parts["gather"] = S * (8 + 4 * K) + B * W * 6
    else:
        W = F * K
        parts["gather"] = gather_bytes(S, K, B, deep)
    if deep:
        g = [(B, H1, W, True, False), (B, H2, H1, False, False),   # fwd0, fwd1
             (B, H1, H2, True, True), (B, W, H1, False, False),    # dH1 (mask aux), dX
             (H2, H1, B, False, False), (H1, W, B, False, False)]  # dW1, dW0
        parts["gemm"] = sum(gemm_planes_bytes(*a) for a in g)
        flops = sum(2.0 * a[0] * a[1] * a[2] for a in g)
        parts["head"] = B * H2 * (4 + 6) + B * 16
        dense = W * H1 + H1 + H1 * H2 + H2 + H2 + 2
        parts["dense_adam"] = dense * 28 + (W * H1 + H1 * H2) * 6
        if kind == "IPNN":  # per-slot gradients through the pair products
            parts["ipnn_backward"] = S * 8 + S * 4 * K * 2 + B * W * 4
    parts["scatter_apply"] = scatter_bytes(S, K, U, deep and kind != "IPNN", apply=True)
    parts["flush_amortised"] = flush_bytes_per_step
    return parts, flops


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def flush_bytes(V, K, lin=True):
    """deferred_flush_tile, algorithmic: read + write p, m, v of every element (24 B) and of
    the linear weight, read + write last[] (8 B per row)."""
    return 24 * V * K + (24 * V if lin else 0) + 8 * V


def host_threads() -> tuple[int, str]:
    """Every core this process may run on (torch.set_num_threads(cpu count)):
    the CPU affinity set, capped by a cgroup CPU quota when one is set (a quota of Q cores
    runs at most Q threads at once; more would only time-slice)."""
    n = len(os.sched_getaffinity(0))
    note = f"sched_getaffinity: {n} cores"
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            q = max(1, int(int(quota) / int(period)))
            note += f"; cgroup cpu.max quota {int(quota) / int(period):g} cores"
            n = min(n, q)
    except (OSError, ValueError):
        pass
    return n, note


def cpu_baseline(cfg, batches, max_seconds=25.0):
    """The oracle (torch-CPU restatement, pinned to the reference) on this host."""
    from oracle import ctr_oracle as O
    threads, thread_note = host_threads()
    torch.set_num_threads(threads)
    t0 = time.perf_counter()
    params = O.init_params(cfg["kind"], cfg["V"], cfg["F"], cfg["K"], seed=1)
    opt = O.make_optimizer(params, 1e-3, 1e-5)
    init_s = time.perf_counter() - t0
    xs = [torch.from_numpy(x) for x, _ in batches]
    ys = [torch.from_numpy(y) for _, y in batches]
    for i in range(2):  # warm-up (allocates the dense grads), BASELINE.md protocol
        O.train_step(cfg["kind"], params, opt, xs[i % len(xs)], ys[i % len(ys)])
    n, t, split = 0, 0.0, {}
    while n < 1 or (t < max_seconds and n < 10):
        s = time.perf_counter()
        O.train_step(cfg["kind"], params, opt, xs[n % len(xs)], ys[n % len(ys)], split=split)
        t += time.perf_counter() - s
        n += 1
        if t > max_seconds / 2 and n >= 3:
            break
    eps = n * cfg["B"] / t
    return {"value": eps, "unit": "examples/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "threads_note": thread_note,
            "split_ms_per_step": {k: v / n * 1e3 for k, v in split.items()},
            "sample": f"{n} timed steps (+2 warm-up) of the same workload and batches on the "
                      f"host CPU, oracle/ctr_oracle.py train_step (torch-CPU ops as the "
                      f"reference: dense nn.Embedding grads, torch.optim.Adam); "
                      f"{t / n * 1e3:.0f} ms/step; param init {init_s:.1f} s untimed"}


def cpu_baseline_pg(cfg, episodes, max_seconds=25.0):
    """PolicyGradient.learn restated on torch-CPU (oracle.pg_learn) on this host."""
    from oracle import ctr_oracle as O
    threads, thread_note = host_threads()
    torch.set_num_threads(threads)
    torch.manual_seed(1)
    V, F, K, A = cfg["V"], cfg["F"], cfg["K"], cfg["A"]
    E = torch.randn(V, K)
    policy = O.pg_policy(F * (F - 1) // 2 + F * K, A)
    opt = torch.optim.Adam(policy.parameters(), lr=1e-4, weight_decay=1e-5)
    eps = [(torch.from_numpy(x), torch.from_numpy(a), r) for x, a, r in episodes]
    O.pg_learn(policy, opt, E, *eps[0])  # warm-up
    n, t = 0, 0.0
    while n < 3 or (t < max_seconds and n < 10):
        s = time.perf_counter()
        O.pg_learn(policy, opt, E, *eps[n % len(eps)])
        t += time.perf_counter() - s
        n += 1
    return {"value": n * cfg["B"] / t, "unit": "transitions/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "threads_note": thread_note,
            "sample": f"{n} timed learn() calls (+1 warm-up) on the same episodes, "
                      f"oracle/ctr_oracle.py pg_learn (torch-CPU: FE state, policy MLP, "
                      f"loss_func, Adam); {t / n * 1e3:.0f} ms per episode"}


def bench_pg(args, cfg, world, rank, dev):
    """C4: one step = store_transition(episode) + learn() (PG_model.py:156-179) on this
    rank's B transitions; N>1 = one episode of N*B transitions split over the ranks."""
    from rl_ctr_prediction_amd import PolicyGradient, hip_ops
    from rl_ctr_prediction_amd.synthetic import CriteoSynth

    V, F, K, B, A = cfg["V"], cfg["F"], cfg["K"], cfg["B"], cfg["A"]
    torch.manual_seed(1)  # identical replicas
    pg = PolicyGradient(V, F, K, "c4", action_nums=A, device=str(dev), fix_input_dims=True)
    pg.policy_net.train()
    synth = CriteoSynth(V, F, seed=1)
    n_eps = max(1, min(args.batches, args.warmup))
    rng = np.random.default_rng([4, rank])
    host = []
    # reward r_b = -BCE(y_b, p_{a_b}) (SURVEY.md §8d's C4 definition; the reference's is
    # commented out, hybrid_td3_main_per_v10.py:147-150): p_{b,a} = the pCTR of candidate
    # model a — synthetic here: the planted FM logit of the batch with a fixed per-action
    # distortion (model a's logit shrunk by 1/(1+0.1a) and shifted by 0.25a)
    for x, y in synth.batches(n_eps, B, rank=rank):
        a = rng.integers(1, A + 1, size=(B, 1)).astype(np.int64)
        z0 = np.log(0.25 / 0.75) + synth.planted_logit(x)
        za = z0[:, None] / (1.0 + 0.1 * np.arange(1, A + 1)) + 0.25 * np.arange(1, A + 1)
        pa = 1.0 / (1.0 + np.exp(-za[np.arange(B), a[:, 0] - 1]))
        yb = y.astype(np.float64)
        bce = -(yb * np.maximum(np.log(pa), -100.0) + (1 - yb) * np.maximum(np.log1p(-pa), -100.0))
        host.append((x, a, (-bce).reshape(-1, 1).astype(np.float32)))
    eps = [tuple(torch.from_numpy(t).to(dev) for t in e) for e in host]

    def step(i):
        x, a, r = eps[i % len(eps)]
        pg.store_transition(x, a, r)
        return pg.learn()

    for i in range(args.warmup):
        step(i)
    # roofline pass (not timed): HIP events around every policy GEMM launch
    spans = []
    real_gemm = hip_ops.gemm

    def timed(fn, flops_of):
        def wrap(*a, **kw):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = fn(*a, **kw)
            e1.record()
            spans.append((e0, e1, flops_of(out, a, kw)))
            return out
        return wrap

    def gemm_flops(res, a, kw):  # hip_ops.gemm(a, b, trans_a, trans_b, ...)
        trans_a = a[2] if len(a) > 2 else kw.get("trans_a", False)
        return 2.0 * res.shape[0] * res.shape[1] * (a[0].shape[0] if trans_a else a[0].shape[1])

    def planes_flops(res, a, kw):  # hip_ops.gemm_planes(A, B, a_rc, b_rc, out=...)
        A, Bp, a_rc, b_rc = a[0], a[1], a[2], a[3]
        M, K = (A.cols, A.rows) if a_rc else (A.rows, A.cols)
        N = Bp.cols if b_rc else Bp.rows
        return 2.0 * M * N * K

    # hip_ops.linear calls hip_ops.gemm through the module, so wrapping gemm sees every launch;
    # the breakdown runs eagerly (a graph replay cannot carry timing events)
    real_planes = hip_ops.gemm_planes
    hip_ops.gemm = timed(real_gemm, gemm_flops)
    hip_ops.gemm_planes = timed(real_planes, planes_flops)
    pg.use_graphs = False
    fe_ev = []
    real_fe = hip_ops.feature_embedding

    def fe_wrap(*a, **kw):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = real_fe(*a, **kw)
        e1.record()
        fe_ev.append((e0, e1))
        return out

    hip_ops.feature_embedding = fe_wrap
    try:
        n_bd = max(1, min(args.steps, args.breakdown_steps))
        for i in range(n_bd):
            step(i)
        torch.cuda.synchronize()
    finally:
        hip_ops.gemm, hip_ops.feature_embedding = real_gemm, real_fe
        hip_ops.gemm_planes = real_planes
        pg.use_graphs = True

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        loss = step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    g_ms = [a.elapsed_time(b) for a, b, _ in spans]
    flops = sum(w for _, _, w in spans) / len(spans)
    launch_ms = sum(g_ms) / len(g_ms)
    achieved = flops / (launch_ms * 1e-3) / 1e12
    fe_ms = sum(a.elapsed_time(b) for a, b in fe_ev) / len(fe_ev)
    fe_bytes = B * F * 8 + B * F * 4 * K + B * (F * (F - 1) // 2 + F * K) * 4
    result = {
        "metric": METRIC, "value": world * B * args.steps / elapsed, "unit": "transitions/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": "synthetic: Criteo-shape ids as states, uniform actions, reward = -BCE(y, "
                "p_a) of the chosen candidate model's pCTR (SURVEY §8d C4); random-init weights",
        "config": {"workload": cfg["workload"], "model": "PolicyGradient (Net, fix_input_dims)",
                   "episode_transitions": B * world, "fields": F, "vocab": V, "embed_dim": K,
                   "actions": A, "parallelism": f"dp{world}" + (
                       " (one episode split over the ranks: reward all-gather, gradient "
                       "all-reduce)" if world > 1 else ""),
                   "optimizer": "Adam lr=1e-4 wd=1e-5 (PG_model.py:87)"},
        "roofline": {"kernel": "policy MLP GEMMs fwd + bwd, averaged per launch "
                               "(gemm_planes_kernel on the 741-1024-512-256 layers, "
                               "ctr_gemm_f32_ex on the 256-128-A tail)",
                     "bound": "mfma", "achieved": achieved, "peak": MFMA_F32_PEAK_TFS,
                     "unit": "TFLOP/s", "frac": achieved / MFMA_F32_PEAK_TFS,
                     "algorithmic_flops_per_launch": flops,
                     "traffic": load_traffic("c4", "gemm")[0],
                     "traffic_source": load_traffic("c4", "gemm")[1],
                     "avg_launch_ms": launch_ms, "launches_timed": len(spans),
                     "timing": "HIP events on the launch stream around each GEMM launch over "
                               "un-timed learn() calls before the timed region"},
        "kernels": {"feature_embedding_kernel": {"ms_per_call": fe_ms,
                                                 "GBps": fe_bytes / (fe_ms * 1e-3) / 1e9},
                    "policy GEMMs": {"ms_per_step": sum(g_ms) / n_bd}},
        "_graphs": "timed region: every learn() replays one HIP graph after the zero-std "
                   "check of the returns (one host sync); breakdown: eager launches",
        "last_loss": float(loss.item()),
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline ...")
        result["cpu_baseline"] = cpu_baseline_pg(cfg, host)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def load_mfma_busy():
    """Matrix-pipe busy fraction of the six MLP GEMMs (rocprofv3 SQ_VALU_MFMA_BUSY_CYCLES
    over the SIMD-cycles of each launch, standalone; profiles/*gemm_mfma_busy.json from
    tools/gemm_planes_pmc.sh), weighted by each launch's cycles."""
    for p in sorted((ROOT / "profiles").glob("*gemm_mfma_busy.json"), reverse=True):
        try:
            d = json.loads(p.read_text())["shapes"]
            busy = sum(v["mfma_busy_cycles"] for v in d.values())
            simd = sum(1024 * v["grbm_gui_active"] / 8 for v in d.values())
            return busy / simd, f"profiles/{p.name}"
        except Exception:
            continue
    return None


def load_crosscal(config: str):
    """The oracle's CPU step time over the reference's own, measured side by side in the
    build container (tools/cpu_crosscal.py -> profiles/*cpu_crosscal.json)."""
    for p in sorted((ROOT / "profiles").glob("*cpu_crosscal.json"), reverse=True):
        try:
            d = json.loads(p.read_text())
            c = d["configs"][config]
            return {"oracle_over_reference": c["oracle_over_reference"],
                    "within_10pct": c["within_10pct"], "threads": d["threads"],
                    "host": d["cpu_model"], "source": f"profiles/{p.name}"}
        except Exception:
            continue
    return None


def load_traffic(config: str, kernel: str):
    """HBM bytes per launch of the dominant kernel from the committed PMC summary (rocprofv3
    FETCH_SIZE/WRITE_SIZE passes with the gfx950 corrections, profiles/)."""
    for p in sorted((ROOT / "profiles").glob("*pmc*.json"), reverse=True):
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        k = d.get(config, {}).get(kernel)
        if k and k.get("hbm_bytes_per_launch"):
            return float(k["hbm_bytes_per_launch"]), p.name
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--batches", type=int, default=0,
                    help="0 (default): a fresh synthetic batch for every step (streaming, as the "
                         "reference trains: all_main/pretrain_main.py:71-78); N > 0: N distinct "
                         "batches cycled")
    ap.add_argument("--flush-every", type=int, default=None,
                    help="deferred Adam: flush every N steps (bounded staleness; default: the "
                         "trainer's, CTR_FLUSH_EVERY or 32; 0 = only at the region end)")
    ap.add_argument("--breakdown-steps", type=int, default=10,
                    help="un-timed steps with every kernel group instrumented (kernel table)")
    ap.add_argument("--sharding", default="auto", choices=["auto", "rows", "replicated"],
                    help="N>1: row-sharded tables with all-to-all (auto) or, for comparison only "
                         "(eager, a host read per step), replicated tables "
                         "with a sparse all-gather")
    ap.add_argument("--lookahead", type=int, default=2,
                    help="sparse plans built this many batches ahead, concurrently with the "
                         "step (FusedCTRTrainer next_x); 0 = every plan in its own step")
    ap.add_argument("--no-stage-labels", action="store_true",
                    help="lookahead stages the next batches' ids only (next_y not passed): "
                         "every step copies its labels on the main stream")
    ap.add_argument("--optimizer", default="deferred", choices=["deferred", "dense"],
                    help="deferred-exact dense Adam (default) or the dense streaming pass; "
                         "bitwise-identical results (tests/test_gpu_deferred.py)")
    ap.add_argument("--no-driver-loop", action="store_true",
                    help="skip the driver-loop measurement (pretrain_main.run_epoch over K "
                         "batches after the timed region)")
    ap.add_argument("--no-graphs", action="store_true",
                    help="launch every step eagerly (no HIP-graph replay): the host-paced "
                         "launch path (N > 1 row sharding over gloo, or CTR_SHARDED_GRAPHS=0)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        log(f"--gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    # CTR_DIST_BACKEND=gloo + more ranks than GPUs: a functional rehearsal of the N>1 path
    # on a one-GPU box (collectives staged through the host; timings meaningless)
    backend = os.environ.get("CTR_DIST_BACKEND", "nccl")
    dev = torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from rl_ctr_prediction_amd import DeepFM, FM, FusedCTRTrainer, InnerPNN, ShardedCTRTrainer
    from rl_ctr_prediction_amd.synthetic import CriteoSynth

    cfg = CONFIGS[args.config]
    if cfg["kind"] == "PG":
        return bench_pg(args, cfg, world, rank, dev)
    V, F, K, B = cfg["V"], cfg["F"], cfg["K"], cfg["B"]
    t0 = time.perf_counter()
    torch.manual_seed(1)  # identical replicas on every rank
    with torch.device(dev):
        model = {"FM": lambda: FM(V, K), "DeepFM": lambda: DeepFM(V, F, K),
                 "IPNN": lambda: InnerPNN(V, F, K)}[cfg["kind"]]()
    model.train()
    synth = CriteoSynth(V, F, seed=1)
    n_bd = max(1, min(args.steps, args.breakdown_steps))
    # streaming (default): every step of the warm-up, the breakdown pass and the timed region
    # trains on a batch of its own (the roofline pass after the region revisits the timed
    # region's batches); the HIP graphs are keyed by input slot, not by batch
    n_batches = args.batches if args.batches > 0 else args.warmup + n_bd + 3 + args.steps
    t_gen = time.perf_counter()
    host_batches = synth.stream(n_batches, B, rank=rank, threads=min(16, os.cpu_count() or 1))
    xs = [torch.from_numpy(x).to(dev) for x, _ in host_batches]
    ys = [torch.from_numpy(y).to(dev) for _, y in host_batches]
    log(f"{n_batches} distinct batches generated in {time.perf_counter() - t_gen:.1f}s")
    sharding = args.sharding
    if sharding == "auto":
        sharding = "rows" if world > 1 and args.optimizer == "deferred" else "replicated"
    if sharding == "rows":
        trainer = ShardedCTRTrainer(model, lr=1e-3, weight_decay=1e-5, seed=1234)
    else:
        trainer = FusedCTRTrainer(model, lr=1e-3, weight_decay=1e-5, seed=1234,
                                  optimizer_mode=args.optimizer)
    if args.no_graphs:
        trainer.use_graphs = False
    if args.flush_every is not None:
        trainer.flush_every = args.flush_every
    log(f"rank {rank}/{world}: {cfg['kind']} V={V} K={K} B={B} ready in {time.perf_counter() - t0:.1f}s")

    # one running batch index over every loop below, so each step's lookahead batch is the
    # batch the next step trains on (the graphs captured in the warm-up are the ones replayed)
    seq = [0]

    def step(_i):
        i = seq[0]
        seq[0] += 1
        nxt = [xs[(i + j) % len(xs)] for j in range(1, args.lookahead + 1)]
        nyt = None if args.no_stage_labels else [ys[(i + j) % len(ys)]
                                                 for j in range(1, args.lookahead + 1)]
        trainer.step(xs[i % len(xs)], ys[i % len(ys)], next_x=nxt, return_loss=False,
                     next_y=nyt)

    for i in range(args.warmup):
        step(i)

    def total_ms(spans):
        return float(sum(a.elapsed_time(b) for a, b, _ in spans))

    def avg_ms(spans):
        return total_ms(spans) / len(spans) if spans else float("nan")

    # breakdown pass (NOT timed): every kernel group bracketed by HIP events, to find the
    # dominant kernel and report the per-kernel table
    keys = ("adam", "catchup", "gather", "plan", "scatter", "flush", "gemm", "exchange")
    trainer.flush()
    trainer.timing = {k: [] for k in keys}
    for i in range(n_bd):
        step(i)
    trainer.flush()
    torch.cuda.synchronize()
    bd, trainer.timing = trainer.timing, None
    per_step = {k: total_ms(v) / n_bd for k, v in bd.items()}
    # N = 1 deferred: the embedding Adam apply runs inside the scatter's combine pass
    fused_apply = (world == 1 and args.optimizer == "deferred" and isinstance(
        trainer, FusedCTRTrainer) and not isinstance(trainer, ShardedCTRTrainer)
        and trainer.fuse_apply and trainer._vec_ok and trainer.K >= 32)
    dominant = max(("adam", "catchup", "gather", "plan", "scatter", "gemm", "flush"),
                   key=lambda k: per_step[k])

    # re-warm (untimed), only with the pipelined weight-gradient tail (CTR_PIPELINE_WGRAD=1):
    # the breakdown's flush left no tail pending; a few graph-replayed steps restore the
    # steady state the timed region runs in (every graph it replays captured before it
    # starts), and a flush after them keeps the region's own flush at K replayed steps
    trainer.timing = None
    if getattr(trainer, "_pipe", False):
        for i in range(3):
            step(i)
        trainer._flush_table()  # the tables only: the tail stays pending
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # timed region: nothing instrumented (at N=1 the steps replay as HIP graphs)
    trainer.timing = None
    captures0 = getattr(trainer, "captures", 0)
    t_start = time.perf_counter()
    host_s = 0.0  # time spent inside step() (enqueueing): the host's share of a step
    for i in range(args.steps):
        t_h = time.perf_counter()
        step(i)
        host_s += time.perf_counter() - t_h
    # deferred mode: every row is brought to the last step INSIDE the timed region, so the
    # measured work is the complete dense-Adam trajectory of K steps (nothing left owed)
    trainer.flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    captures_region = getattr(trainer, "captures", 0) - captures0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # roofline pass: the same K steps again, launched eagerly with HIP events recorded on
    # the launch stream around every launch of the dominant kernel group (a HIP graph
    # cannot carry timing events: hipErrorInvalidHandle); kernel durations do not depend
    # on how the kernel was launched, and the rocprofv3 trace of the graph-replayed run
    # (profiles/) is the cross-check
    trainer.timing = {dominant: [], "flush": [], "catchup": []}
    for i in range(args.steps):
        step(i)
    trainer.flush()
    torch.cuda.synchronize()
    timing = trainer.timing
    trainer.timing = None

    # the driver's own loop (pretrain_main.train -> run_epoch: lookahead steps, the loss
    # summed on the device and read once), and the reference's per-step `.item()` loop for
    # comparison, each over K batches + the flush, N = 1 (pretrain_main is one process)
    driver = None
    if world == 1 and not args.no_driver_loop:
        from rl_ctr_prediction_amd.pretrain_main import run_epoch
        base = seq[0]
        dl = [(xs[(base + j) % len(xs)], ys[(base + j) % len(ys)]) for j in range(args.steps)]
        trainer.flush()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mean_loss = run_epoch(trainer, dl)
        trainer.flush()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        t0 = time.perf_counter()
        tot = 0.0
        for j, (x_j, y_j) in enumerate(dl):
            nxt = [b[0] for b in dl[j + 1:j + 3]]
            tot += trainer.step(x_j, y_j, next_x=nxt, next_y=[b[1] for b in dl[j + 1:j + 3]]).item()
        trainer.flush()
        torch.cuda.synchronize()
        dt_item = time.perf_counter() - t0
        driver = {"value": B * args.steps / dt, "unit": "examples/s",
                  "ms_per_step": dt / args.steps * 1e3, "mean_loss": mean_loss,
                  "item_per_step": {"value": B * args.steps / dt_item,
                                    "ms_per_step": dt_item / args.steps * 1e3,
                                    "mean_loss": tot / args.steps},
                  "what": "pretrain_main.run_epoch (the driver's train() loop: step() with the "
                          "next two batches' plans built ahead, each step's loss added to a "
                          "device float64 sum, read once) over K batches + the flush; "
                          "item_per_step: the same steps with the reference's per-step "
                          "`total_loss += loss.item()` host sync (all_main/pretrain_main.py:79)"}

    U = trainer._bufs.plan.num_unique_host()
    S = B * F
    deep = cfg["kind"] in MLP_KINDS
    gemm_flops_bd = sum(w for _, _, w in bd["gemm"])
    kernels = {
        "_note": f"breakdown pass of {n_bd} un-timed steps (+flush), every group bracketed "
                 f"by HIP events; ms per step",
        "adam_rows" if args.optimizer == "deferred" else "adam_embedding_vec":
            {"ms_per_step": per_step["adam"]},
        "catch-up (deferred rows of the batch replayed before the forward)": {
            "ms_per_step": per_step["catchup"],
            "ms_per_step_after_region": total_ms(timing["catchup"]) / args.steps,
            "_note": "second figure: the roofline pass's K eager steps right after the timed "
                     "region (staleness as deep as the region's flushes allow)"},
        "flush (deferred_flush_tile, once per region)": {"ms_per_step": per_step["flush"]},
        "_graphs": "timed region: HIP-graph replay of the whole step (N=1); breakdown and "
                   "roofline passes: eager launches with HIP events",
        "MLP GEMMs (gemm_planes_kernel + split-K reduce, fwd+bwd)": {
            "ms_per_step": per_step["gemm"],
            "TFLOP/s": gemm_flops_bd / (total_ms(bd["gemm"]) * 1e-3) / 1e12 if bd["gemm"] else None},
        "gather (fm_forward_vec)": {"ms_per_step": per_step["gather"]},
        "sparse plan (column plan: per-field LDS sorts + merge)": {"ms_per_step": per_step["plan"]},
        "scatter (fm_embedding_grad segmented sums)": {"ms_per_step": per_step["scatter"]},
        "exchange (RCCL collectives + row gathers, N>1)": {"ms_per_step": per_step["exchange"]},
    }
    spans = timing[dominant]
    launch_ms = avg_ms(spans)
    if dominant == "gemm":
        flops = sum(w for _, _, w in spans) / len(spans)
        achieved = flops / (launch_ms * 1e-3) / 1e12
        roofline = {"kernel": "MLP GEMMs (gemm_planes_kernel: fp32-accurate split-bf16 MFMA on "
                              "pre-split operand planes, + split-K reduce), the 6 of a step "
                              "averaged per launch",
                    "bound": "mfma", "achieved": achieved, "peak": MFMA_F32_PEAK_TFS,
                    "unit": "TFLOP/s", "frac": achieved / MFMA_F32_PEAK_TFS,
                    "peak_note": "fp32 matrix peak (the path's dtype; achieved = 2*M*N*K / "
                                 "launch time); the split-bf16 algorithm issues 6 bf16 MFMA "
                                 "products per fp32 product: bf16_mfma_frac = 6*achieved / "
                                 "2500 TF bf16 dense",
                    "bf16_mfma_frac": 6.0 * achieved / MFMA_BF16_PEAK_TFS,
                    "algorithmic_flops_per_launch": flops}
        busy = load_mfma_busy()
        if busy is not None:
            roofline["mfma_busy"], roofline["mfma_busy_source"] = busy
        traffic, src = load_traffic(args.config, "gemm")
    else:
        if dominant in ("adam", "catchup"):
            if args.optimizer == "dense":
                nbytes = adam_bytes(V, K, U)
                kname = "adam_embedding_vec (dense Adam over E[V,K] + w[V])"
            else:  # catch-up or apply of the batch's U rows: read+write p,m,v (+grad rows)
                nbytes = U * 24 * (K + 1) + U * (4 * K + 8) // 2
                kname = "deferred_rows_vec (catch-up / apply of the batch's rows, per launch)"
        elif dominant == "flush":
            nbytes = flush_bytes(trainer.V_tab, K, lin=trainer.w_tab is not None)
            kname = ("deferred_flush_tile (every row of the table brought to the region's last "
                     "step, once per timed region)")
        elif dominant == "gather":
            nbytes, kname = ((ipnn_gather_bytes(S, K, B, F), "ipnn_forward_kernel")
                             if cfg["kind"] == "IPNN" else
                             (gather_bytes(S, K, B, deep), "fm_forward_vec (embedding gather + FM)"))
        elif dominant == "scatter":
            nbytes = scatter_bytes(S, K, U, deep, apply=fused_apply)
            kname = ("seg_chunk_kernel + seg_combine_apply_kernel (per-row gradient sums with "
                     "the deferred Adam apply fused)" if fused_apply else
                     "seg_chunk_kernel + seg_combine_kernel (per-row gradient sums)")
        else:
            nbytes = plan_bytes(S, U)
            kname = "sparse plan (colplan_sort + colplan_merge + seg_write)"
        achieved = nbytes / (launch_ms * 1e-3) / 1e9
        roofline = {"kernel": kname, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                    "algorithmic_bytes_per_launch": nbytes}
        # the kernels of the dominant group, one launch of each (their PMC traffic summed)
        parts = {"plan": ["colplan_sort_kernel", "colplan_merge_kernel", "seg_write_kernel"],
                 "scatter": ["seg_chunk_kernel", "seg_combine_apply_kernel" if fused_apply
                             else "seg_combine_kernel"],
                 "catchup": ["deferred_rows_vec"],
                 "gather": ["ipnn_forward_kernel" if cfg["kind"] == "IPNN" else "fm_forward_vec"],
                 "adam": ["adam_embedding_vec"],
                 "flush": ["deferred_flush_tile"]}[dominant]
        got = [load_traffic(args.config, k) for k in parts]
        traffic = sum(t for t, _ in got) if all(t for t, _ in got) else None
        src = got[0][1] if traffic else None
        if traffic is not None and len(parts) > 1:
            roofline["traffic_kernels"] = parts
    roofline.update({"traffic": traffic, "traffic_source": src, "avg_launch_ms": launch_ms,
                     "launches_timed": len(spans),
                     "timing": "HIP events on the launch stream around each launch of this "
                               "kernel over K eager steps right after the timed region"})
    kernels["flush (deferred_flush_tile, every flush_every steps and at the region end)"] = \
        kernels.pop("flush (deferred_flush_tile, once per region)")
    kernels["flush (deferred_flush_tile, every flush_every steps and at the region end)"].update(
        region_of_K_steps_ms_total=total_ms(timing["flush"]), flushes=len(timing["flush"]))
    gather_ms, scatter_ms = avg_ms(bd["gather"]), avg_ms(bd["scatter"])
    if cfg["kind"] == "IPNN":
        g_kernel, g_bytes = "ipnn_forward_kernel (gather + pair dots -> MLP input)", \
            ipnn_gather_bytes(S, K, B, F)
    else:
        g_kernel, g_bytes = "fm_forward_vec (gather + FM" + (
            ", MLP input as bf16 planes)" if deep else ")"), gather_bytes(S, K, B, deep)
    value = world * B * args.steps / elapsed
    # the step against the machine: every byte and flop of the algorithm the region times
    # (deferred-exact dense Adam; the flushes inside the region amortised over its steps)
    n_flush = len(timing["flush"])
    fb = flush_bytes(trainer.V_tab, K, lin=trainer.w_tab is not None) * n_flush / args.steps
    parts, sflops = step_model(cfg["kind"], B, F, K, U, flush_bytes_per_step=fb,
                               lin=trainer.w_tab is not None)
    sbytes = sum(parts.values())
    step_s = elapsed / args.steps
    step_roofline = {
        "bytes_per_step": sbytes, "flops_per_step": sflops,
        "hbm_GBps": sbytes / step_s / 1e9, "hbm_frac": sbytes / step_s / 1e9 / HBM_PEAK_GBS,
        "mfma_TFps": sflops / step_s / 1e12 if sflops else None,
        "mfma_frac": sflops / step_s / 1e12 / MFMA_F32_PEAK_TFS if sflops else None,
        "bound_ms": max(sbytes / (HBM_PEAK_GBS * 1e9), sflops / (MFMA_F32_PEAK_TFS * 1e12)) * 1e3,
        "serial_bound_ms": (sbytes / (HBM_PEAK_GBS * 1e9)
                            + sflops / (MFMA_F32_PEAK_TFS * 1e12)) * 1e3,
        "parts_bytes": parts, "unique_rows": U, "flushes_in_region": n_flush,
        "model": "algorithmic bytes of the deferred-exact step (bench.step_model, DESIGN.md §5):"
                 " plan + catch-up of the U batch rows + gather/forward + MLP GEMMs (planes) +"
                 " head + row sums with the fused Adam apply + dense Adam + the region's "
                 "flushes / K; flops = the six MLP GEMMs; hbm_frac / mfma_frac over the "
                 "timed ms_per_step, bound_ms = max(bytes/8 TB/s, flops/157.3 TF)"}
    if world > 1:
        step_roofline["_note"] = "N > 1: per rank; the exchange's bytes are not in the model"
    result = {
        "metric": METRIC, "value": value, "unit": "examples/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (Criteo-shape ids: skewed field cardinalities, Zipf(1.1); "
                "planted-FM labels, CTR~0.25); random-init weights",
        "config": {"workload": cfg["workload"], "model": cfg["kind"], "global_batch": B * world,
                   "fields": F, "vocab": V, "embed_dim": K,
                   "parallelism": f"dp{world}" + (
                       " (row-sharded tables: ids/rows/row-grads by all-to-all, dense grads "
                       "all-reduce)" if sharding == "rows" else
                       " (replicated tables, sparse row-grad all-gather)" if world > 1 else ""),
                   "optimizer": f"dense Adam lr=1e-3 wd=1e-5 (reference semantics), "
                                f"{args.optimizer} mode",
                   "batches": ("fresh: one synthetic batch per step" if args.batches <= 0
                               else f"{args.batches} distinct, cycled"),
                   "flush_every": getattr(trainer, "flush_every", None),
                   "plan_lookahead": (args.lookahead if isinstance(trainer, ShardedCTRTrainer)
                                      or (getattr(trainer, "plan_lookahead", False)
                                          and args.optimizer == "deferred") else 0)},
        "roofline": roofline,
        "step_roofline": step_roofline,
        "kernels": kernels,
        "host_ms_per_step": host_s / args.steps * 1e3,  # inside step(): the enqueue cost
        "graph_captures": {"total": getattr(trainer, "captures", None),
                           "in_timed_region": captures_region,
                           "graphs_held": len(getattr(trainer, "_graphs", {}))},
        "driver_loop": driver,
        "gather_scatter": {
            "gather_kernel": g_kernel, "gather_ms": gather_ms,
            "gather_GBps": g_bytes / (gather_ms * 1e-3) / 1e9,
            "scatter_kernels": ("seg_chunk_kernel + seg_combine_apply_kernel (per-row sums "
                                "and the fused deferred-Adam apply of the batch's rows"
                                if fused_apply else
                                "seg_chunk_kernel + seg_combine_kernel (per-row sums") +
                               "; the sparse plan is timed separately under kernels)",
            "scatter_ms": scatter_ms,
            "scatter_GBps": scatter_bytes(S, K, U, deep, apply=fused_apply)
            / (scatter_ms * 1e-3) / 1e9,
            "unique_rows_per_batch": U, "slots_per_batch": S},
        "cpu_baseline": None,
    }
    if isinstance(trainer, ShardedCTRTrainer):
        # the row-sharded exchange as it ran: this rank's shard, the agreed capacity C (rows
        # per (requester, owner) pair) and the bytes each collective moves per step
        from rl_ctr_prediction_amd import hip_ops as H
        C = int(trainer._cap)
        lin = trainer.w_tab is not None
        chunk = H.rows_chunk(C, K, lin)
        dense_n = int(trainer.flat_grad.numel())
        result["sharding"] = {
            # rows: ["cyclic", rank, N, V] (this rank owns global rows rank::N) or, for the
            # blocks layout, [row_lo, row_hi, V] (sharded.shard_meta)
            "shard_rows": int(trainer.V_tab), "layout": trainer.layout,
            "rows": trainer.shard_meta(),
            "capacity_rows": C, "chunk_floats": int(chunk),
            "exchange_bytes_per_step": {
                "ids_alltoall": world * C * 4, "rows_alltoall": world * chunk * 4,
                "grads_alltoall": world * chunk * 4,
                "dense_allreduce": (dense_n + 1) * 4},
            "unique_rows_this_batch": U,
            "padding_frac": 1.0 - U / max(1, world * C),
            "backend": dist.get_backend() if world > 1 else None,
            "graphs": bool(trainer.use_graphs and trainer._graph_ok),
            "captures": getattr(trainer, "captures", None),
            "host_reads_blocking": trainer.cap_blocking, "host_reads": trainer.cap_reads}
        if world > 1:  # every rank's shard and capacity, gathered to rank 0 for the line
            mine = [trainer.V_tab, trainer.shard_meta(), C, U]
            allr = [None] * world
            dist.all_gather_object(allr, mine)
            result["sharding"]["per_rank"] = [
                {"rank": r, "shard_rows": a[0], "rows": a[1], "capacity_rows": a[2],
                 "unique_rows_last_batch": a[3]} for r, a in enumerate(allr)]
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline ...")
        result["cpu_baseline"] = cpu_baseline(cfg, host_batches)
        cc = load_crosscal(args.config)
        if cc is not None:  # how the port's CPU time compares with the reference's own
            result["cpu_baseline"]["cross_calibration"] = cc
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
