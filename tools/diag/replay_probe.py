"""Diagnostic (GPU box): how much do the two utterance-group graphs of GraphedTranscriber(streams=2)
overlap on the device, and what does the host spend launching them?

Per form, REPS replays after warm-up, timed two ways: host time of the replay calls
(time.perf_counter around them) and device time (events on the caller's stream around the whole
batch of replays, every stream joined back).  Forms:
  g0 / g1     one group's graph alone (on its usual stream)
  both        GraphedTranscriber.step() (group 0 on the caller's stream, group 1 on its own)
  serial      group 0 then group 1, both on the caller's stream
  one         GraphedTranscriber(streams=1): one graph of the whole batch

usage: replay_probe.py [B] [REPS]
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "velocity-asr_amd"))
import torch

import velocity_asr as va
from velocity_asr import synthetic as S
from velocity_asr.pipeline import GraphedTranscriber

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 50
dev = torch.device("cuda", 0)
m = va.VELOCITYASR()
m.load_state_dict({k: torch.from_numpy(v) for k, v in S.make_weights(None, seed=0).items()}, strict=True)
m = m.to(dev).eval()
audio = torch.from_numpy(S.make_audio(B, 160000, seed=1234)).to(dev)
tr2 = GraphedTranscriber(m, B, 160000, streams=2)
tr1 = GraphedTranscriber(m, B, 160000, streams=1)
tr2.audio.copy_(audio)
tr1.audio.copy_(audio)
main = torch.cuda.current_stream(dev)
s1 = tr2.streams[1]


def g0():
    tr2.graphs[0].replay()


def g1():
    s1.wait_stream(main)
    with torch.cuda.stream(s1):
        tr2.graphs[1].replay()
    main.wait_stream(s1)


def serial():
    tr2.graphs[0].replay()
    tr2.graphs[1].replay()


def delayed(cycles):
    def f():
        s1.wait_stream(main)
        tr2.graphs[0].replay()
        with torch.cuda.stream(s1):
            torch.cuda._sleep(cycles)
            tr2.graphs[1].replay()
        main.wait_stream(s1)
    return f


# both groups in ONE graph captured on two streams (fork at the start, join at the end): does
# the runtime run a graph's independent branches concurrently?
from velocity_asr.pipeline import audio_to_token_ids  # noqa: E402
G = B // 2
fa, fb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
o_tok = torch.zeros((B, 501), device=dev, dtype=torch.int32)
o_len = torch.zeros((B,), device=dev, dtype=torch.int32)
fj = torch.cuda.CUDAGraph()
with torch.cuda.graph(fj, stream=fa):
    fb.wait_stream(fa)
    audio_to_token_ids(m, tr2.audio[:G], out=(o_tok[:G], o_len[:G]))
    with torch.cuda.stream(fb):
        audio_to_token_ids(m, tr2.audio[G:], out=(o_tok[G:], o_len[G:]))
    fa.wait_stream(fb)

FORMS = dict(g0=g0, g1=g1, both=tr2.step, serial=serial, one=tr1.step, forkjoin=fj.replay)
for cyc in (20000, 50000, 100000, 200000, 400000):
    FORMS[f"d{cyc // 1000}k"] = delayed(cyc)


def sleep_only(cyc):
    def f():
        torch.cuda._sleep(cyc)
    return f


FORMS["sleep100k"] = sleep_only(100000)
for name, fn in FORMS.items():
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    host = 0.0
    a.record()
    for _ in range(REPS):
        t = time.perf_counter()
        fn()
        host += time.perf_counter() - t
    b.record()
    torch.cuda.synchronize()
    print(f"{name:7s} device {a.elapsed_time(b) / REPS * 1e3:8.1f} us/replay   host {host / REPS * 1e6:8.1f} us/replay",
          flush=True)
# host cost of one graph's replay call alone, with the device idle in between
for name, gr in (("g0 idle", tr2.graphs[0]), ("one idle", tr1.graphs[0])):
    hs = []
    for _ in range(20):
        torch.cuda.synchronize()
        t = time.perf_counter()
        gr.replay()
        hs.append(time.perf_counter() - t)
    torch.cuda.synchronize()
    hs.sort()
    print(f"{name:8s} host replay call: median {hs[10] * 1e6:.1f} us, min {hs[0] * 1e6:.1f} us", flush=True)
