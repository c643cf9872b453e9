"""Phase times inside the column plan's sort kernel (tuning build with CTR_COLPLAN_TRACE=1):

    python tools/build_variant.py cptrace sparse_plan.hip -DCTR_COLPLAN_TRACE=1
    CTR_HIP_LIB=rl_ctr_prediction_amd/variants/lib_cptrace.so python tools/colplan_trace.py

Builds the C2 / C3 plans a few times, then reads each sort block's wall_clock64 marks (100 MHz:
10 ns ticks) and prints per config the block medians and maxima of: ids loaded + range
reduced, each radix pass, the run write-out, and the launch span (first start to last end).
"""
from __future__ import annotations

import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    import bench
    from rl_ctr_prediction_amd import hip_ops as H
    from rl_ctr_prediction_amd._lib import lib
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    fn = lib.raw("ctr_debug_colplan_trace")
    fn.argtypes = [C.c_void_p, C.c_int]
    fn.restype = C.c_int
    dev = torch.device("cuda:0")
    for name in ("c2", "c3"):
        cfg = bench.CONFIGS[name]
        V, F, B = cfg["V"], cfg["F"], cfg["B"]
        x = torch.from_numpy(next(CriteoSynth(V, F, seed=1).batches(1, B))[0]).to(dev)
        P = H.SparsePlanBuffers(B * F, dev)
        for _ in range(5):
            P.build(x, V)
        torch.cuda.synchronize()
        buf = np.zeros((F, 8), dtype=np.uint64)
        assert fn(buf.ctypes.data, F) == 0
        t = buf[:, :6].astype(np.int64)
        bits = buf[:, 6].astype(np.int64)
        passes = (bits + 7) // 8
        ph = {"load_reduce": t[:, 1] - t[:, 0]}
        prev = t[:, 1]
        for k in range(3):
            has = passes > k
            ph[f"pass{k + 1}"] = np.where(has, t[:, 2 + k] - prev, 0)
            prev = np.where(has, t[:, 2 + k], prev)
        ph["write"] = t[:, 5] - prev
        ph["block"] = t[:, 5] - t[:, 0]
        out = {"config": name, "blocks": F, "bits": bits.tolist(),
               "span_us": float(t[:, 5].max() - t[:, 0].min()) / 100.0,
               "start_skew_us": float(t[:, 0].max() - t[:, 0].min()) / 100.0}
        for k, v in ph.items():
            out[k + "_us"] = {"med": float(np.median(v)) / 100.0, "max": float(v.max()) / 100.0}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
