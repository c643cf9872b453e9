"""Diagnostic: padded vs variable-split row-sharded exchange at world size 2 (gloo, one
GPU), per step: which table rows differ, between which runs (each protocol run twice to
separate a race from a systematic difference)."""
import os
import socket
import sys

import numpy as np
import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, kind, K, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "tests"))
    from test_gpu_sharded import _model
    torch.cuda.set_device(0)
    V, F, B, steps = 40_000, 26, 512, 5
    data = [(torch.tensor(x[rank * B:(rank + 1) * B], device="cuda:0"),
             torch.tensor(y[rank * B:(rank + 1) * B], device="cuda:0"))
            for x, y in CriteoSynth(V, F, seed=23).batches(steps, B * world)]
    out = {}
    for run in ("padded", "varsplit", "varsplit", "padded", "varsplit", "varsplit",
                "padded-noahead"):
        m = _model(kind, V, F, K, drop=0.2)
        ex = run.split("-")[0]
        tr = P.ShardedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=3, exchange=ex)
        rec = []
        for i, (xs, ys) in enumerate(data):
            ahead = run.endswith("noahead")
            nxt = None if ahead else ([d[0] for d in data[i + 1:i + 3]] if (rank + i) % 3 else None)
            loss = tr.step(xs, ys, next_x=nxt).item()
            E, w = tr.gather_tables()
            rec.append((loss, E.cpu().numpy(), None if w is None else w.cpu().numpy()))
        key = run
        while key in out:
            key += "'"
        out[key] = rec
    if rank == 0:
        hot = set(np.unique(np.concatenate([x.ravel() for x, _ in
                                            CriteoSynth(V, F, seed=23).batches(steps, B * world)])))
        names = list(out)
        for a in range(len(names)):
            for b in range(a + 1, len(names)):
                A, Bb = out[names[a]], out[names[b]]
                msg = []
                for s in range(len(A)):
                    dE = np.nonzero((A[s][1] != Bb[s][1]).any(1))[0]
                    dw = (np.nonzero((A[s][2] != Bb[s][2]).ravel())[0]
                          if A[s][2] is not None else [])
                    if len(dE) or len(dw) or A[s][0] != Bb[s][0]:
                        msg.append(f"step{s}: loss {'=' if A[s][0] == Bb[s][0] else '!='} "
                                   f"E rows {len(dE)} {list(dE[:8])} w {len(dw)} "
                                   f"max|dE| {np.abs(A[s][1] - Bb[s][1]).max():.3g}")
                print(kind, K, names[a], "vs", names[b], "equal" if not msg else "; ".join(msg),
                      flush=True)
    q.put(rank)
    dist.destroy_process_group()


if __name__ == "__main__":
    for kind, K in (("FM", 32), ("DeepFM", 16)):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _port()
        ps = [ctx.Process(target=_rank, args=(r, 2, port, kind, K, q)) for r in range(2)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(timeout=300)
            if p.exitcode != 0:
                print("rank failed", p.exitcode)
                sys.exit(1)
