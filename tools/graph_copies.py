"""What runs inside one graphed step: capture a GraphedTranscriber
(B clips x S samples, `streams` utterance groups), then replay it REPS times between two
marker kernels (torch.cuda._sleep -> spin_kernel), under `rocprofv3 --kernel-trace`.

  python3 tools/graph_copies.py [B] [S] [streams]          (under rocprofv3, GPU box)
  python tools/graph_copies.py --summary <kernel_trace.csv>  (anywhere)

The summary lists, per kernel name, launches and mean duration per step, then the step's
timeline: wall span per replay, summed kernel time, and the idle gaps between consecutive
kernels (launch / dependency latency of the graph)."""
import collections
import csv
import os
import sys

REPS = 10


def run(B=32, S=160000, streams=2):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "velocity-asr_amd"))
    import torch

    import velocity_asr as va
    from velocity_asr import synthetic as Syn
    from velocity_asr.pipeline import GraphedTranscriber

    dev = torch.device("cuda", 0)
    W = Syn.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = m.to(dev).eval()
    tr = GraphedTranscriber(m, B, S, dev, streams=streams)
    tr.audio.copy_(torch.from_numpy(Syn.make_audio(B, S, seed=1234)).to(dev))
    tr.step()
    torch.cuda.synchronize()
    torch.cuda._sleep(100000)  # marker
    torch.cuda.synchronize()
    for _ in range(REPS):
        tr.step()
        torch.cuda.synchronize()  # one replay at a time: each step's span is its latency
    torch.cuda._sleep(100000)  # marker
    torch.cuda.synchronize()
    print("replayed", REPS)


def short(name):
    n = name.replace("void ", "").replace("vasr::(anonymous namespace)::", "")
    return n.split("(")[0][:70]


def summary(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]]
    a, b = marks[-2], marks[-1]
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows[a + 1:b]]
    cnt = collections.Counter(k[2] for k in ks)
    dur = collections.defaultdict(float)
    for s, e, n in ks:
        dur[n] += (e - s) / 1e3
    print(f"{'launches/step':>13} {'us/launch':>9} {'us/step':>8}  kernel")
    for n, c in cnt.most_common():
        print(f"{c / REPS:13.2f} {dur[n] / c:9.2f} {dur[n] / REPS:8.2f}  {n}")
    # per-step timeline: steps are separated by the host synchronize (the largest gaps)
    gaps = sorted(((ks[i + 1][0] - ks[i][1], i) for i in range(len(ks) - 1)), reverse=True)[:REPS - 1]
    cuts = sorted(i for _, i in gaps)
    steps, lo = [], 0
    for c in cuts + [len(ks) - 1]:
        steps.append(ks[lo:c + 1])
        lo = c + 1
    spans, busy, idle = [], [], []
    for st in steps:
        t0, t1 = st[0][0], max(e for _, e, _ in st)
        spans.append((t1 - t0) / 1e3)
        # union of kernel intervals (overlapping streams count once)
        cov, cur_s, cur_e = 0, None, None
        for s, e, _ in sorted(st):
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    cov += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        cov += cur_e - cur_s
        busy.append(cov / 1e3)
        idle.append((t1 - t0 - cov) / 1e3)
    n = len(steps)
    print(f"\nper replay (device side, {n} replays): span {sum(spans) / n:.1f} us, kernels busy {sum(busy) / n:.1f} us, "
          f"idle gaps {sum(idle) / n:.1f} us, {len(ks) / n:.0f} launches")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        summary(sys.argv[2])
    else:
        run(*[int(v) for v in sys.argv[1:4]])
