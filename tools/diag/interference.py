"""Diagnostic (GPU box): which kernel, running concurrently on another stream, corrupts another
kernel's output?  (r04a: with two utterance groups in flight -- graphs or eager -- group 1's
first kernel, the |STFT|^2 launch, sometimes ends with different values in a few clips.)

Every ops call of one eager pass over group 0 (16 clips) is recorded with its arguments; each
recorded op type in turn is the aggressor: REPS launches of it on stream A while stream B runs
REPS launches of the victim (each into its own output), host-interleaved so the two streams'
kernels overlap on the device.  Each victim output is compared bitwise with the victim run
alone.  Victims: the STFT of group 1's audio, and the scan of group 1's first local block.

usage: interference.py [REPS]
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

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 30
dev = torch.device("cuda", 0)
NAMES = ("gemm", "gemm_argmax", "layer_norm", "ln_dwconv", "ssm_scan", "ssm_block_tail", "adaptive_pool",
         "pooled_attention", "stft_power_400", "mel_log_norm", "ctc_collapse", "add_table")
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
    audio_to_token_ids(m, a0)  # builds the cached layouts
    calls = []
    audio_to_token_ids(m, a0)  # first call of every op type, with its arguments
    rec, calls = calls, None
torch.cuda.synchronize()
print("aggressors:", len(rec), flush=True)

tb = A._tables(dev, 400, 80, 16000)
with torch.no_grad():
    blk = m.local_ssm.layers[0]
    mel1 = A.mel_on_device(a1, frame_pad=1)
    x1 = m.temporal_binding(mel1).contiguous()
    B1, L1, D1 = x1.shape
    u1 = orig["ln_dwconv"](x1, blk.norm1.weight, blk.norm1.bias, blk.conv.weight.view(D1, -1), blk.conv.bias,
                           blk.norm1.eps).view(B1 * L1, D1)
    xz1, xdt1 = blk.ssm.project(u1)
victims = {
    "stft": lambda: orig["stft_power_400"](a1, tb.window),
    "scan": lambda: blk.ssm.scan(xz1, xdt1, B1, L1),
}
for vkey in os.environ.get("VICTIMS", "").split(";"):  # extra victims: recorded group-0 calls by key prefix
    for name, fn, a, k in rec:
        if vkey and name.startswith(vkey):
            victims[name] = (lambda fn=fn, a=a, k=k: fn(*a, **k))
            break
only = os.environ.get("ONLY_VICTIMS")
if only:
    victims = {n: v for n, v in victims.items() if any(n.startswith(o) for o in only.split(";"))}


def bits(t):
    t = t[0] if isinstance(t, tuple) else t
    return t.contiguous().view(torch.int32) if t.dtype == torch.float32 else t.contiguous()


aggs = os.environ.get("AGGRESSORS")
if aggs:
    rec = [c for c in rec if any(c[0].startswith(a) for a in aggs.split(";"))]
ref = {k: bits(v()).clone() for k, v in victims.items()}
torch.cuda.synchronize()
sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
main = torch.cuda.current_stream(dev)
for vname, victim in victims.items():
    for agg in [("none", None, (), {})] + rec:
        aname, fn, a, k = agg
        outs = []
        sa.wait_stream(main)
        sb.wait_stream(main)
        with torch.no_grad():
            for _ in range(REPS):
                if fn is not None:
                    with torch.cuda.stream(sa):
                        fn(*a, **k)
                with torch.cuda.stream(sb):
                    outs.append(victim())
        main.wait_stream(sa)
        main.wait_stream(sb)
        torch.cuda.synchronize()
        bad = [i for i, o in enumerate(outs) if not torch.equal(bits(o), ref[vname])]
        nel = [int((bits(outs[i]) != ref[vname]).sum()) for i in bad[:5]]
        print(f"victim {vname:5s} aggressor {aname:48s}: {len(bad)}/{REPS} corrupted {bad[:8]} elements {nel}", flush=True)
        if bad and os.environ.get("DETAIL") and vname == "scan":
            for i in bad[:3]:
                g, r_ = outs[i].contiguous(), ref[vname].view(torch.float32)
                idx = (bits(g) != ref[vname]).nonzero()
                rows, cols = idx[:, 0], idx[:, 1]
                bb, tt = rows // L1, rows % L1
                print(f"   rep {i}: {len(idx)} elements; clips {sorted(set(bb.tolist()))}; steps {tt.min().item()}..{tt.max().item()} "
                      f"chunks32 {sorted(set((tt // 32).tolist()))}; channels {sorted(set(cols.tolist()))[:24]}", flush=True)
                for j in range(min(6, len(idx))):
                    a_, c_ = rows[j].item(), cols[j].item()
                    print(f"     b={a_ // L1} t={a_ % L1} d={c_}: got {g[a_, c_].item():.6e} ref {r_[a_, c_].item():.6e}", flush=True)
        del outs
