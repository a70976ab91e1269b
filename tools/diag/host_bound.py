"""Diagnostic (GPU box): is the bench's step paced by the device or by the host's graph launches?
For the C2 batch (32 x 10 s, one graph): the host time of one hipGraphLaunch (CUDAGraph.replay) and
of GraphedTranscriber.step (replay + parameter check), and the device time per step when
  (a) the host launches step after step (the bench's timed loop),
  (b) the queue is filled ahead first (REPS replays enqueued while the device is held busy by a
      spin kernel, so the device never waits on the host),
plus the same for one 10-s utterance.  usage: host_bound.py"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "velocity-asr_amd"))
import torch  # noqa: E402

import velocity_asr as va  # noqa: E402
from velocity_asr import ops  # noqa: E402
from velocity_asr import synthetic as S  # noqa: E402
from velocity_asr.pipeline import GraphedTranscriber  # noqa: E402

dev = torch.device("cuda", 0)
m = va.VELOCITYASR()
m.load_state_dict({k: torch.from_numpy(v) for k, v in S.make_weights(None, seed=0).items()}, strict=True)
m = m.to(dev).eval()
REPS = 40
for B, secs in ((32, 10.0), (1, 10.0)):
    tr = GraphedTranscriber(m, B, int(secs * 16000), dev, streams=1)
    tr.audio.copy_(torch.from_numpy(S.make_audio(B, int(secs * 16000), seed=1234)).to(dev))
    for _ in range(10):
        tr.step()
    torch.cuda.synchronize()
    # host cost of one replay call, the device idle (each replay waits for the previous to end)
    hr, hs = [], []
    for _ in range(REPS):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.graphs[0].replay()
        hr.append(time.perf_counter() - t0)
    for _ in range(REPS):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.step()
        hs.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    # (a) host launches step after step
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    t0 = time.perf_counter()
    for _ in range(REPS):
        tr.step()
    t_issue = time.perf_counter() - t0
    b.record()
    torch.cuda.synchronize()
    dev_a = a.elapsed_time(b) / REPS
    # (b) queue filled ahead: hold the device with a clock probe launch long enough for the host to
    # enqueue every replay, then time the replays alone (events after the probe)
    hold = torch.zeros(3 * 2048, device=dev, dtype=torch.int64)
    from velocity_asr import _lib
    _lib.check(_lib.load().vasr_probe_clock(hold.data_ptr(), 2048, 16_000_000, torch.cuda.current_stream(dev).cuda_stream),
               "vasr_probe_clock")
    a.record()
    for _ in range(REPS):
        tr.step()
    b.record()
    torch.cuda.synchronize()
    dev_b = a.elapsed_time(b) / REPS
    med = lambda v: sorted(v)[len(v) // 2] * 1e3  # noqa: E731
    print(f"B={B:2d} {secs:.0f} s: host per replay() {med(hr):.3f} ms, per step() {med(hs):.3f} ms; "
          f"device per step: host-paced {dev_a:.3f} ms (loop issue {t_issue / REPS * 1e3:.3f} ms/step), "
          f"queue filled ahead {dev_b:.3f} ms", flush=True)
    del tr
    torch.cuda.synchronize()
