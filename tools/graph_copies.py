"""Which kernels run inside the graphed bench step: capture the bench's
GraphedTranscriber (32 x 10 s, two utterance groups), then replay it REPS times between two
marker kernels (torch.cuda._sleep), under `rocprofv3 --kernel-trace`.  Summarise with
`python tools/graph_copies.py --summary <kernel_trace.csv>`: per kernel name, the launches
between the markers divided by REPS.
Usage (GPU box): rocprofv3 --kernel-trace -d gpurun_out/gc -o run --output-format csv -- \
    python3 tools/graph_copies.py"""
import collections
import csv
import os
import sys

REPS = 10


def run():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "velocity-asr_amd"))
    import torch

    import velocity_asr as va
    from velocity_asr import synthetic as S
    from velocity_asr.pipeline import GraphedTranscriber

    dev = torch.device("cuda", 0)
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = m.to(dev).eval()
    tr = GraphedTranscriber(m, 32, 160000, dev, streams=2)
    tr.audio.copy_(torch.from_numpy(S.make_audio(32, 160000, seed=1234)).to(dev))
    tr.step()
    torch.cuda.synchronize()
    torch.cuda._sleep(100000)  # marker
    torch.cuda.synchronize()
    for _ in range(REPS):
        tr.step()
    torch.cuda.synchronize()
    torch.cuda._sleep(100000)  # marker
    torch.cuda.synchronize()
    print("replayed", REPS)


def summary(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]]
    a, b = marks[-2], marks[-1]
    cnt = collections.Counter(r["Kernel_Name"][:100] for r in rows[a + 1:b])
    for k, v in cnt.most_common():
        print(f"{v / REPS:8.2f}  {k}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        summary(sys.argv[2])
    else:
        run()
