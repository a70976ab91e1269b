"""Diagnostic (GPU box): GraphedTranscriber(2 clips, 2 utterance groups) built repeatedly and
replayed with the audio rewritten before each step; tokens vs the eager result.  Mode "caller":
group 0 on the caller's stream (HEAD); mode "own": every group on its own stream (events both ways)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "velocity-asr_amd"))
import torch
import velocity_asr as va
from velocity_asr import synthetic as S
from velocity_asr.pipeline import GraphedTranscriber, audio_to_token_ids, token_lists

mode = sys.argv[1] if len(sys.argv) > 1 else "caller"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2
NB, REPS = int(os.environ.get("STRESS_NB", 16)), int(os.environ.get("STRESS_REPS", 25))  # builds, replays per build
dev = torch.device("cuda", 0)
m = va.VELOCITYASR()
m.load_state_dict({k: torch.from_numpy(v) for k, v in S.make_weights(None, seed=0).items()}, strict=True)
m = m.to(dev).eval()
audio = torch.from_numpy(S.make_audio(B, 160000, seed=1234)).to(dev)
with torch.no_grad():
    exp = token_lists(*audio_to_token_ids(m, audio))


def step_own(tr):
    main = torch.cuda.current_stream(dev)
    for st in tr.streams:
        st.wait_stream(main)
    for st, gr in zip(tr.streams, tr.graphs):
        with torch.cuda.stream(st):
            gr.replay()
    for st in tr.streams:
        main.wait_stream(st)


def step_seq(tr):
    main = torch.cuda.current_stream(dev)
    prev = main
    for st, gr in zip(tr.streams, tr.graphs):
        st.wait_stream(prev)
        with torch.cuda.stream(st):
            gr.replay()
        prev = st
    main.wait_stream(prev)


streams = 1 if mode == "single" else 2
bad = []
for b in range(NB):
    tr = GraphedTranscriber(m, B, 160000, dev, streams=streams)
    for r in range(REPS):
        tr.audio.zero_()
        tr.audio.copy_(audio)
        if mode == "own":
            step_own(tr)
        elif mode == "seq":
            step_seq(tr)
        else:
            tr.step()
        got = token_lists(*tr.collect())
        if got != exp:
            bad.append((b, r, [i for i in range(B) if got[i] != exp[i]]))
    del tr
    print(f"build {b}: mismatches so far {len(bad)}", flush=True)
print("MODE", mode, "B", B, "replays", NB * REPS, "mismatching replays", len(bad), bad[:10], flush=True)
