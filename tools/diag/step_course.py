"""Diagnostic (GPU box): the time course of the C2 step (32 x 10 s, one graph) within a burst of
back-to-back steps, under different histories -- why the bench's first timed steps run up to 25 %
slower than its last (profiles/r05h/, r05i/).
  A  40 steps right after 20 warm steps (deep queue: the host enqueues all of them at once)
  B  the same after 0.5 s idle
  C  40 steps with a device synchronize after each (queue depth 1)
  D  40 steps without events between them (total only)
  E  80 steps after 0.5 s idle (does the course settle, and where)
usage: step_course.py"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "velocity-asr_amd"))
import torch  # noqa: E402

import velocity_asr as va  # noqa: E402
from velocity_asr import synthetic as S  # noqa: E402
from velocity_asr.pipeline import GraphedTranscriber  # noqa: E402

dev = torch.device("cuda", 0)
m = va.VELOCITYASR()
m.load_state_dict({k: torch.from_numpy(v) for k, v in S.make_weights(None, seed=0).items()}, strict=True)
m = m.to(dev).eval()
tr = GraphedTranscriber(m, 32, 160000, dev, streams=1)
tr.audio.copy_(torch.from_numpy(S.make_audio(32, 160000, seed=1234)).to(dev))


def burst(n, sync_each=False, events=True):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        if events:
            ev[i].record()
        tr.step()
        if sync_each:
            torch.cuda.synchronize()
    if events:
        ev[n].record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n * 1e3
    return wall, ([ev[i].elapsed_time(ev[i + 1]) for i in range(n)] if events else [])


def show(tag, r):
    wall, ms = r
    s = f"{tag}: wall {wall:.3f} ms/step"
    if ms:
        q = len(ms) // 4
        s += (f"; device ms first 8 {[round(v, 3) for v in ms[:8]]}, quarter means "
              f"{[round(sum(ms[i * q:(i + 1) * q]) / q, 3) for i in range(4)]}, last {ms[-1]:.3f}")
    print(s, flush=True)


burst(20)
show("A deep queue after 20 warm", burst(40))
time.sleep(0.5)
show("B after 0.5 s idle", burst(40))
show("C synchronize after each step", burst(40, sync_each=True))
show("D no events (wall only)", burst(40, events=False))
time.sleep(0.5)
show("E 80 steps after 0.5 s idle", burst(80))
show("F 80 more, right after", burst(80))
