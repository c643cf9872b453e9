"""Cross-calibrate bench.py's CPU baseline (the oracle, `kind: "port"`) against the
reference itself, on this container's CPU (build container only: the reference never
travels to the GPU box).

    PYTHONDONTWRITEBYTECODE=1 python tools/cpu_crosscal.py [--steps 4] [--threads 8]

For C2 (FM, 1M x 16, batch 4096) and C3 (DeepFM, 10M x 64, batch 8192): the reference's
own training step (src/all_main/pretrain_main.py:67-79: model(x), nn.BCELoss, zero_grad,
backward, torch.optim.Adam.step, imported from /root/reference, nothing copied) and the
oracle's train_step (oracle/ctr_oracle.py) on the same synthetic batches, same thread
count, alternating A/B per step. Writes profiles/r02_cpu_crosscal.json with the per-step
medians and the ratio oracle / reference; BASELINE.md asks for agreement within +-10 %.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
REF = Path(os.environ.get("CTR_REFERENCE", "/root/reference"))
sys.path.insert(0, str(ROOT))

from oracle import ctr_oracle as O  # noqa: E402
from rl_ctr_prediction_amd.synthetic import CriteoSynth  # noqa: E402

CFGS = {"c2": dict(kind="FM", V=1_000_000, F=26, K=16, B=4096),
        "c3": dict(kind="DeepFM", V=10_000_000, F=26, K=64, B=8192)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    args = ap.parse_args()
    if not REF.exists():
        raise SystemExit(f"{REF} not found: run in the build container")
    sys.dont_write_bytecode = True
    sys.path.insert(0, str(REF))
    import src.models.p_model as P  # noqa: E402  (the reference, imported read-only)
    torch.set_num_threads(args.threads)
    out = {"threads": args.threads, "steps": args.steps, "cpu_model": _cpu_model(),
           "torch": torch.__version__, "configs": {}}
    for name, c in CFGS.items():
        batches = list(CriteoSynth(c["V"], c["F"], seed=3).batches(2, c["B"]))
        xs = [torch.from_numpy(x).long() for x, _ in batches]
        ys = [torch.from_numpy(y).float() for _, y in batches]
        torch.manual_seed(1)
        ref = (P.FM(c["V"], c["K"]) if c["kind"] == "FM"
               else P.DeepFM(c["V"], c["F"], c["K"]))
        for mod in ref.modules():  # both paths without dropout: same arithmetic per step
            if isinstance(mod, torch.nn.Dropout):
                mod.p = 0.0
        ref.train()
        r_opt = torch.optim.Adam(params=ref.parameters(), lr=1e-3, weight_decay=1e-5)
        loss_fn = torch.nn.BCELoss()
        params = O.init_params(c["kind"], c["V"], c["F"], c["K"], seed=1)
        o_opt = O.make_optimizer(params, 1e-3, 1e-5)

        def ref_step(i):
            y = ref(xs[i % 2])
            loss = loss_fn(y, ys[i % 2].reshape(-1, 1))
            ref.zero_grad()
            loss.backward()
            r_opt.step()
            return loss.item()

        def oracle_step(i):
            return O.train_step(c["kind"], params, o_opt, xs[i % 2], ys[i % 2], drop_p=0.0)

        ref_step(0)  # warm-up: allocates the dense gradients and Adam state
        oracle_step(0)
        tr, to = [], []
        for i in range(1, args.steps + 1):
            s = time.perf_counter()
            ref_step(i)
            tr.append(time.perf_counter() - s)
            s = time.perf_counter()
            oracle_step(i)
            to.append(time.perf_counter() - s)
        mr, mo = statistics.median(tr), statistics.median(to)
        out["configs"][name] = {
            "workload": f"{c['kind']} V={c['V']} K={c['K']} B={c['B']} F={c['F']}",
            "reference_ms_per_step": mr * 1e3, "oracle_ms_per_step": mo * 1e3,
            "reference_ex_per_s": c["B"] / mr, "oracle_ex_per_s": c["B"] / mo,
            "oracle_over_reference": mo / mr, "within_10pct": abs(mo / mr - 1.0) <= 0.10,
            "ref_all_ms": [t * 1e3 for t in tr], "oracle_all_ms": [t * 1e3 for t in to]}
        print(name, json.dumps(out["configs"][name]), flush=True)
        del ref, r_opt, params, o_opt
    (ROOT / "profiles" / "r02_cpu_crosscal.json").write_text(json.dumps(out, indent=1) + "\n")


def _cpu_model() -> str:
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            return line.split(":", 1)[1].strip()
    return "unknown"


if __name__ == "__main__":
    main()
