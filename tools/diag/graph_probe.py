"""Diagnostic (GPU box): locate the first kernel output that differs when two utterance-group
graphs replay concurrently.

Every ops wrapper's returned tensor is recorded ("probes") while capturing each group's graph;
the probe tensors stay referenced, so after a replay they hold that replay's values.  The
reference values come from an eager pass of the same group (same kernels, same shapes, so
bitwise equal when nothing races).  After every concurrent replay the probes of both groups are
compared bitwise with the references and the first differing probe is reported with the rows
that differ.

usage: graph_probe.py MODE [B] [BUILDS] [REPS]
  MODE graph   two graphs, group 0 on the caller's stream, group 1 on its own (GraphedTranscriber)
       own     two graphs, each on its own stream
       eager   no graphs: the two groups' eager passes issued on two streams concurrently
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "velocity-asr_amd"))
import torch

import velocity_asr as va
from velocity_asr import ops
from velocity_asr import synthetic as S
from velocity_asr.pipeline import audio_to_token_ids, token_lists

mode = sys.argv[1] if len(sys.argv) > 1 else "graph"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
BUILDS = int(sys.argv[3]) if len(sys.argv) > 3 else 8
REPS = int(sys.argv[4]) if len(sys.argv) > 4 else 25
G = B // 2
dev = torch.device("cuda", 0)

_probe = None
_WRAPPED = ("gemm", "gemm_argmax", "layer_norm", "ln_dwconv", "ssm_scan", "ssm_block_tail", "adaptive_pool",
            "pooled_attention", "stft_power_400", "mel_log_norm", "ctc_collapse", "add_table")


def _wrap(name, fn):
    def w(*a, **k):
        out = fn(*a, **k)
        if _probe is not None:
            outs = out if isinstance(out, tuple) else (out,)
            for i, t in enumerate(outs):
                if isinstance(t, torch.Tensor):
                    _probe.append((f"{name}#{len(_probe)}" + (f".{i}" if len(outs) > 1 else ""), t))
        return out
    return w


for n in _WRAPPED:
    setattr(ops, n, _wrap(n, getattr(ops, n)))

m = va.VELOCITYASR()
m.load_state_dict({k: torch.from_numpy(v) for k, v in S.make_weights(None, seed=0).items()}, strict=True)
m = m.to(dev).eval()
audio_all = torch.from_numpy(S.make_audio(B, 160000, seed=1234)).to(dev)


def bits(t):
    t = t.contiguous()
    return t.view(torch.int32) if t.dtype == torch.float32 else t


def eager_probes(x):
    global _probe
    _probe = []
    with torch.no_grad():
        audio_to_token_ids(m, x)
    torch.cuda.synchronize()
    out, _probe = [(n, bits(t).clone()) for n, t in _probe], None
    return out


with torch.no_grad():
    exp = token_lists(*audio_to_token_ids(m, audio_all))
ref = [eager_probes(audio_all[g * G:(g + 1) * G].contiguous()) for g in range(2)]
print("probes per group", len(ref[0]), flush=True)


def first_diff(probes, refs):
    for (n, t), (_, r) in zip(probes, refs):
        if n.startswith("ctc_collapse") and n.endswith(".0"):
            continue  # token rows past each clip's length are never written (stale, not compared)
        b = bits(t)
        if b.shape != r.shape:
            return n, "shape", None
        d = b != r
        if bool(d.any()):
            flat = d.reshape(d.shape[0], -1).any(1).nonzero().flatten()
            rows = flat.tolist()
            if os.environ.get("DETAIL"):
                idx = d.reshape(-1).nonzero().flatten()
                got_v = t.contiguous().reshape(-1)[idx[:12]].tolist()
                ref_v = r.view(torch.float32).reshape(-1)[idx[:12]].tolist() if t.dtype == torch.float32 else []
                runs = (idx[1:] - idx[:-1] != 1).sum().item() + 1
                print(f"   {n}: flat {idx[:12].tolist()} .. {idx[-1].item()} ({runs} runs); got {got_v}; ref {ref_v}; "
                      f"base {t.data_ptr():#x}", flush=True)
                # where else does each wrong value occur bitwise in the references (either group)?
                pos = [i for i, (pn, _) in enumerate(probes) if pn == n][0]
                for e in idx[:4].tolist():
                    gv = b.reshape(-1)[e]
                    hits = []
                    for gg in range(2):
                        rr = ref[gg][pos][1].reshape(-1)
                        w = (rr == gv).nonzero().flatten()[:4].tolist()
                        hits += [(gg, x) for x in w]
                    print(f"     elem {e}: got bits found at (group, flat) {hits}", flush=True)
            return n, int(d.sum()), (rows[0], rows[-1], len(rows), tuple(t.shape))
    return None


bad, first_stage = [], {}
for b in range(BUILDS):
    audio = torch.zeros((B, 160000), device=dev)
    audio.copy_(audio_all)
    tokens = torch.zeros((B, 501), device=dev, dtype=torch.int32)
    lengths = torch.zeros((B,), device=dev, dtype=torch.int32)
    views = [audio[g * G:(g + 1) * G] for g in range(2)]
    outs = [(tokens[g * G:(g + 1) * G], lengths[g * G:(g + 1) * G]) for g in range(2)]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    main = torch.cuda.current_stream(dev)
    probes = [None, None]
    graphs = []
    if mode != "eager":
        for st, v in zip(streams, views):
            st.wait_stream(main)
            with torch.cuda.stream(st):
                for _ in range(2):
                    audio_to_token_ids(m, v)
            main.wait_stream(st)
        for g, (st, v, o) in enumerate(zip(streams, views, outs)):
            gr = torch.cuda.CUDAGraph()
            _probe = []
            with torch.cuda.graph(gr, stream=st):
                audio_to_token_ids(m, v, out=o)
            probes[g], _probe = _probe, None
            graphs.append(gr)
        if b == 0:
            for g in range(2):
                lo = min(t.data_ptr() for _, t in probes[g])
                hi = max(t.data_ptr() + t.untyped_storage().nbytes() for _, t in probes[g])
                print(f"group {g} probe span {lo:#x}..{hi:#x}", flush=True)
            if os.environ.get("DETAIL"):  # every probe's extent, both groups, sorted by address
                ext = sorted((t.data_ptr(), t.data_ptr() + t.numel() * t.element_size(), g, n)
                             for g in range(2) for n, t in probes[g])
                for a0, a1, g, n in ext:
                    print(f"   extent {a0:#x}..{a1:#x} g{g} {n}", flush=True)
    for r in range(REPS):
        if mode == "graph":
            streams[1].wait_stream(main)
            graphs[0].replay()
            with torch.cuda.stream(streams[1]):
                graphs[1].replay()
            main.wait_stream(streams[1])
        elif mode == "own":
            for st in streams:
                st.wait_stream(main)
            for st, gr in zip(streams, graphs):
                with torch.cuda.stream(st):
                    gr.replay()
            for st in streams:
                main.wait_stream(st)
        else:  # eager: both groups issued on two streams, interleaved by the host
            pr = [[], []]
            for st in streams:
                st.wait_stream(main)
            for g, (st, v, o) in enumerate(zip(streams, views, outs)):
                _probe = pr[g]
                with torch.cuda.stream(st), torch.no_grad():
                    audio_to_token_ids(m, v, out=o)
                _probe = None
            for st in streams:
                main.wait_stream(st)
            probes = pr
        torch.cuda.synchronize()
        got = token_lists(tokens, lengths)
        diffs = [first_diff(probes[g], ref[g]) for g in range(2)]
        if got != exp or any(diffs):
            clips = [i for i in range(B) if got[i] != exp[i]]
            bad.append((b, r, clips, diffs))
            for d in diffs:
                if d:
                    first_stage[d[0]] = first_stage.get(d[0], 0) + 1
            print(f"build {b} rep {r}: clips {clips} first diff g0 {diffs[0]} g1 {diffs[1]}", flush=True)
    del graphs
    print(f"build {b}: mismatching replays so far {len(bad)}", flush=True)
print("MODE", mode, "B", B, "replays", BUILDS * REPS, "mismatching", len(bad), "first stages", first_stage, flush=True)
