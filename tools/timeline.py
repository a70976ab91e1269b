#!/usr/bin/env python3
"""Timeline of a rocprofv3 --kernel-trace run (diagnostic): per-queue busy time, gaps between
consecutive kernels on a queue, and how the queues overlap, over the last `--window` ms of the
trace (the bench's timed steps sit at the end of the run).

Usage: tools/timeline.py gpurun_out/<dir>/trace/run_kernel_trace.csv [--window MS] [--steps K]
"""

import argparse
import collections
import csv
import re


def fam(name):
    n = name.replace("void ", "").replace("vasr::(anonymous namespace)::", "")
    n = re.sub(r"^npl[24]::", "", n.split("(")[0])
    if n.startswith("ssm_scan_kernel"):
        return "scan"
    if n.startswith("gemm_x3_kernel"):
        return "gemm"
    if n.startswith("ssm_tail"):
        return "tail"
    return n.split("<")[0][:28]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--window", type=float, default=0.0, help="ms at the end of the trace (0: steps)")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), fam(r["Kernel_Name"]))
          for r in rows]
    ks.sort()
    t_end = max(k[1] for k in ks)
    if a.window > 0:
        t0 = t_end - a.window * 1e6
    else:
        # the timed steps: the last `steps` collapse kernels end each step of each group
        col = sorted(k[1] for k in ks if k[3] == "collapse_kernel")
        per = len([1 for k in ks if k[3] == "collapse_kernel"])
        t0 = col[-2 * a.steps - 1] if len(col) > 2 * a.steps else ks[0][0]
        t_end = col[-1]
    ks = [k for k in ks if k[0] >= t0 and k[1] <= t_end]
    span = t_end - t0
    queues = sorted(set(k[2] for k in ks))
    print(f"window {span / 1e3:.1f} us, {len(ks)} kernels, queues {queues}")
    for q in queues:
        qk = [k for k in ks if k[2] == q]
        busy = sum(k[1] - k[0] for k in qk)
        gaps = [qk[i + 1][0] - qk[i][1] for i in range(len(qk) - 1)]
        pos = [g for g in gaps if g > 0]
        print(f"queue {q}: {len(qk)} kernels, busy {busy / span:.3f} of the window, "
              f"gaps: total {sum(pos) / 1e3:.1f} us, median {sorted(pos)[len(pos) // 2] / 1e3 if pos else 0:.2f} us, "
              f"overlapping-own {sum(1 for g in gaps if g < 0)}")
        fb = collections.Counter()
        for k in qk:
            fb[k[3]] += k[1] - k[0]
        print("   " + ", ".join(f"{f} {v / span:.3f}" for f, v in fb.most_common(8)))
    # overlap: sweep over events, count busy queues and the pair of families running
    ev = []
    for k in ks:
        ev.append((k[0], 1, k))
        ev.append((k[1], -1, k))
    ev.sort(key=lambda e: (e[0], e[1]))
    active = []
    last = t0
    nbusy = collections.Counter()
    pairs = collections.Counter()
    for t, kind, k in ev:
        dtm = t - last
        if dtm > 0:
            nq = len(set(x[2] for x in active))
            nbusy[nq] += dtm
            if nq >= 2:
                pairs[tuple(sorted(set(x[3] for x in active)))] += dtm
            elif nq == 1:
                pairs[("alone",) + tuple(sorted(set(x[3] for x in active)))] += dtm
        last = t
        if kind == 1:
            active.append(k)
        else:
            active.remove(k)
    print("queues busy at once: " + ", ".join(f"{n}: {v / span:.3f}" for n, v in sorted(nbusy.items())))
    print("time by concurrent kernel families:")
    for p, v in pairs.most_common(16):
        print(f"   {v / span:.3f}  {' + '.join(p)}")


if __name__ == "__main__":
    main()
