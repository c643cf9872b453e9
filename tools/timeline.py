"""Per-step kernel timeline from a rocprofv3 --kernel-trace csv.

    python tools/timeline.py run_kernel_trace.csv [--step N] [--marker step_end_kernel]

Splits the trace at each launch of the marker kernel (one per training step), prints the
kernels of step N (default: the median-length step) with start offset, duration and queue,
then per step: wall time, the time at least one kernel was running (busy) and the gaps.
"""
import argparse
import csv
import re
import statistics


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)  # drop the argument list
    name = name.replace("void ", "").replace("ctr::", "")
    if "at::native" in name:
        return "torch:" + name.split("at::native::")[-1][:40]
    return name[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=None)
    ap.add_argument("--marker", default="step_end_kernel")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         r["Queue_Id"], short(r["Kernel_Name"])))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if a.marker in r[3]]
    if len(starts) < 2:
        raise SystemExit(f"fewer than two '{a.marker}' launches in the trace")
    steps = []
    for j in range(len(starts) - 1):
        seg = rows[starts[j]:starts[j + 1]]
        t0 = seg[0][0]
        t1 = rows[starts[j + 1]][0]
        busy, cur_s, cur_e = 0, None, None
        for s, e, _, _ in seg:
            e = min(e, t1)
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        steps.append((j, t0, t1, busy, seg))
    walls = [s[2] - s[1] for s in steps]
    pick = a.step if a.step is not None else sorted(range(len(steps)), key=lambda i: walls[i])[len(steps) // 2]
    j, t0, t1, busy, seg = steps[pick]
    print(f"step {j}: wall {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
    print(f"{'start':>8} {'dur':>7} {'end':>8}  q  kernel")
    for s, e, q, n in seg:
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {(e - t0) / 1e3:8.1f} {q:>2}  {n}")
    print()
    print("per step: wall / busy (us), kernels launched")
    for j, t0, t1, busy, sg in steps:
        print(f"  {j:3d} {(t1 - t0) / 1e3:8.1f} {busy / 1e3:8.1f} {len(sg):5d}")
    print(f"median wall {statistics.median(walls) / 1e3:.1f} us, "
          f"median kernels per step {statistics.median(len(s[4]) for s in steps)}")


if __name__ == "__main__":
    main()
