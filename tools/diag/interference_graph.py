"""Diagnostic (GPU box): interference matrix with both sides captured as HIP graphs, so the two
streams' kernels really overlap (host-issued eager launches of short kernels barely do).

Every ops call of one eager pass over group 0 (16 clips) is recorded with its arguments (one per
op type and shape).  For each aggressor: graph A = REPS launches of it; graph V = REPS launches of
the victim, each into its own output (kept).  A and V replay on two streams at once; every victim
output is compared bitwise with the victim run alone.  Victims (VICTIMS, ';'-separated): stft
(group 1's |STFT|^2), scan (group 1's first local-block scan), or a recorded key prefix.

usage: interference_graph.py [REPS] [ROUNDS]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "velocity-asr_amd"))
import torch

import velocity_asr as va
from velocity_asr import audio as A
from velocity_asr import ops
from velocity_asr import synthetic as S
from velocity_asr.pipeline import audio_to_token_ids

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
NAMES = ("gemm", "gemm_argmax", "gemm_batched", "layer_norm", "ln_dwconv", "ssm_scan", "ssm_block_tail",
         "adaptive_pool", "pooled_attention", "stft_power_400", "mel_log_norm", "ctc_collapse", "add_table")
calls = None
orig = {n: getattr(ops, n) for n in NAMES}


def _key(name, a):
    shapes = [tuple(t.shape) for t in a[:2] if isinstance(t, torch.Tensor)]
    return f"{name}{shapes}"


def _wrap(name, fn):
    def w(*a, **k):
        if calls is not None and _key(name, a) not in [c[0] for c in calls]:
            calls.append((_key(name, a), fn, a, k))
        return fn(*a, **k)
    return w


for n in NAMES:
    setattr(ops, n, _wrap(n, orig[n]))

m = va.VELOCITYASR()
m.load_state_dict({k: torch.from_numpy(v) for k, v in S.make_weights(None, seed=0).items()}, strict=True)
m = m.to(dev).eval()
audio = torch.from_numpy(S.make_audio(32, 160000, seed=1234)).to(dev)
a0, a1 = audio[:16], audio[16:]
with torch.no_grad():
    audio_to_token_ids(m, a0)
    calls = []
    audio_to_token_ids(m, a0)
    rec, calls = calls, None
torch.cuda.synchronize()
aggs = os.environ.get("AGGRESSORS")
if aggs:
    rec = [c for c in rec if any(c[0].startswith(x) for x in aggs.split(";"))]

tb = A._tables(dev, 400, 80, 16000)
with torch.no_grad():
    blk = m.local_ssm.layers[0]
    mel1 = A.mel_on_device(a1, frame_pad=1)
    x1 = m.temporal_binding(mel1).contiguous()
    B1, L1, D1 = x1.shape
    u1 = orig["ln_dwconv"](x1, blk.norm1.weight, blk.norm1.bias, blk.conv.weight.view(D1, -1), blk.conv.bias,
                           blk.norm1.eps).view(B1 * L1, D1)
    xz1, xdt1 = blk.ssm.project(u1)
victims = {"stft": lambda: orig["stft_power_400"](a1, tb.window), "scan": lambda: blk.ssm.scan(xz1, xdt1, B1, L1)}
only = os.environ.get("VICTIMS", "stft")
victims = {n: v for n, v in victims.items() if n in only.split(";")}


def bits(t):
    t = t[0] if isinstance(t, tuple) else t
    return t.contiguous().view(torch.int32) if t.dtype == torch.float32 else t.contiguous()


def capture(fn, reps, keep):
    st = torch.cuda.Stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(st):
        fn()  # warm
    torch.cuda.current_stream(dev).wait_stream(st)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=st):
        for _ in range(reps):
            out = fn()
            if keep:
                keep.append(out)
    return gr


with torch.no_grad():
    ref = {k: bits(v()).clone() for k, v in victims.items()}
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    main = torch.cuda.current_stream(dev)
    for vname, victim in victims.items():
        outs = []
        gv = capture(victim, REPS, outs)
        for aname, fn, a, k in [("none", None, (), {})] + rec:
            ga = capture(lambda: fn(*a, **k), REPS, None) if fn is not None else None
            bad = 0
            for _ in range(ROUNDS):
                sa.wait_stream(main)
                sb.wait_stream(main)
                if ga is not None:
                    with torch.cuda.stream(sa):
                        ga.replay()
                with torch.cuda.stream(sb):
                    gv.replay()
                main.wait_stream(sa)
                main.wait_stream(sb)
                torch.cuda.synchronize()
                for o in outs:
                    if torch.equal(bits(o), ref[vname]):
                        continue
                    bad += 1
                    if bad <= 2 and vname == "stft":
                        idx = (bits(o) != ref[vname]).nonzero()
                        cl, fr, bn = idx[:, 0], idx[:, 1], idx[:, 2]
                        print(f"   {len(idx)} elements: clips {sorted(set(cl.tolist()))}, frames "
                              f"{sorted(set(fr.tolist()))[:16]}, bins {sorted(set(bn.tolist()))[:24]}", flush=True)
            print(f"victim {vname:5s} aggressor {aname:48s}: {bad}/{REPS * ROUNDS} corrupted", flush=True)
            del ga
