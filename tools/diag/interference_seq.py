"""Diagnostic (GPU box): which prefix of group 0's pipeline, replayed as a graph beside a graph of
group 1's |STFT|^2 launches, changes the STFT outputs?  (r04j: with two full-pipeline graphs
replayed concurrently, group 1's first kernel -- the STFT -- sometimes ends with perturbed
spectra in its first or last clips; no single op replayed beside it does that, r04i.)

Every ops call of one eager pass over group 0 is recorded in order with its arguments; the
aggressor graph is calls[:k] (each re-run on the recorded inputs), the victim graph REPS STFT
launches of group 1's audio, each into its own output.  The aggressor replays on the caller's
stream and the victim right after on its own stream (the GraphedTranscriber order).

usage: interference_seq.py [REPS] [ROUNDS] [SEL ...]
  SEL  k      the prefix calls[:k]
       i,j,.. those recorded calls, in that order (a single index needs a trailing comma: "2,")
env VICTIM=i   the victim is recorded call i (re-run on its recorded inputs) instead of the STFT
env DETAIL=1   the pattern of the first corrupted STFT outputs: per 6-frame block, its frames and bins mod 8
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

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 10
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 10
SELS = sys.argv[3:] or ["1", "2", "4", "5", "6", "8", "12", "20", "40", "1000"]
dev = torch.device("cuda", 0)
NAMES = ("gemm", "gemm_argmax", "gemm_batched", "layer_norm", "ln_dwconv", "ssm_scan", "ssm_block_tail",
         "adaptive_pool", "pooled_attention", "stft_power_400", "mel_log_norm", "ctc_collapse", "add_table")
calls = None
orig = {n: getattr(ops, n) for n in NAMES}


def _wrap(name, fn):
    def w(*a, **k):
        if calls is not None:
            calls.append((name, fn, a, k))
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
print("recorded calls:", len(rec), [c[0] for c in rec[:12]], flush=True)
tb = A._tables(dev, 400, 80, 16000)


def bits(t):
    t = t[0] if isinstance(t, tuple) else t
    return t.contiguous().view(torch.int32) if t.dtype == torch.float32 else t.contiguous()


VIC = os.environ.get("VICTIM")
HSACO = os.environ.get("VICTIM_HSACO")
if HSACO:
    # the victim is stft_power_400_kernel<6> from a standalone code object (tools/diag/stft_surgery.py),
    # launched with hipModuleLaunchKernel on the current (capturing) stream into a fresh output
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    _mod, _fn = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipModuleLoad(ctypes.byref(_mod), HSACO.encode()) == 0, "hipModuleLoad"
    _sym = os.environ.get("VICTIM_SYMBOL", "_ZN4vasr12_GLOBAL__N_121stft_power_400_kernelILi6EEEvPKfliPKiiS3_Pfll")
    assert hip.hipModuleGetFunction(ctypes.byref(_fn), _mod, _sym.encode()) == 0, "hipModuleGetFunction"
    print("victim: module", HSACO, flush=True)
    _keep = []

    def victim():
        B, S = a1.shape
        F = S // 160 + 1
        power = torch.empty((B, F, 201), device=dev, dtype=torch.float32)
        args = [ctypes.c_void_p(a1.data_ptr()), ctypes.c_int64(S), ctypes.c_int32(S), ctypes.c_void_p(0),
                ctypes.c_int32(F), ctypes.c_void_p(tb.window.data_ptr()), ctypes.c_void_p(power.data_ptr()),
                ctypes.c_int64(201), ctypes.c_int64(F * 201)]
        params = (ctypes.c_void_p * len(args))(*[ctypes.cast(ctypes.byref(v), ctypes.c_void_p) for v in args])
        _keep.append((args, params))
        st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        rc = hip.hipModuleLaunchKernel(_fn, (F + 5) // 6, B, 1, 256, 1, 1, 0, st, params, None)
        assert rc == 0, f"hipModuleLaunchKernel {rc}"
        return power
    _lib_ref = orig["stft_power_400"](a1, tb.window)
    _mod_out = victim()
    torch.cuda.synchronize()
    _d = (_mod_out - _lib_ref).abs().max().item()
    print(f"module kernel alone vs the library kernel: max |diff| {_d:.3g}, bitwise equal "
          f"{bool(torch.equal(_mod_out.view(torch.int32), _lib_ref.view(torch.int32)))}", flush=True)
elif VIC is None:
    def victim():
        return orig["stft_power_400"](a1, tb.window)
else:
    _vn, _vf, _va, _vk = rec[int(VIC)]
    print("victim: recorded call", VIC, _vn, flush=True)

    def victim():
        return _vf(*_va, **_vk)


def detail(o):
    """The corrupted elements of one STFT output by workgroup (clip, 6-frame block)."""
    d = bits(o) != ref
    idx = d.nonzero()
    got, want = o.reshape(-1)[d.reshape(-1)], ref.view(torch.float32).reshape(-1)[d.reshape(-1)]
    rel = ((got - want).abs() / want.abs().clamp_min(1e-6)).max().item()
    blocks = {}
    for c, f, b in idx.tolist():
        e = blocks.setdefault((c, f // 6), [set(), set(), 0])
        e[0].add(f % 6)
        e[1].add(b % 8)
        e[2] += 1
    items = sorted(blocks.items())
    print(f"   {len(idx)} elements in {len(blocks)} workgroups, max rel err {rel:.3g}; first: "
          + "; ".join(f"c{c} b{bx} q{sorted(qs)} k%8{sorted(ks)} n{n}" for (c, bx), (qs, ks, n) in items[:10]),
          flush=True)


def capture(fn, keep=None, reps=1):
    st = torch.cuda.Stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(st):
        fn()
    torch.cuda.current_stream(dev).wait_stream(st)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=st):
        for _ in range(reps):
            out = fn()
            if keep is not None:
                keep.append(out)
    return gr


shown = 0
with torch.no_grad():
    ref = bits(victim()).clone()
    outs = []
    gv = capture(victim, outs, REPS)
    sv = torch.cuda.Stream(dev)
    main = torch.cuda.current_stream(dev)
    for spec in SELS:
        if "," in spec:
            idx = [int(v) for v in spec.split(",") if v]
            sel, label = [rec[i] for i in idx], f"calls {idx}"
        else:
            sel = rec[:int(spec)]
            label = f"calls[:{len(sel)}]"

        def agg():
            for name, fn, a, kw in sel:
                fn(*a, **kw)
        ga = capture(agg)
        bad, clips, launches = 0, set(), {}
        for _ in range(ROUNDS):
            sv.wait_stream(main)
            ga.replay()  # the caller's stream, as GraphedTranscriber replays group 0
            with torch.cuda.stream(sv):
                gv.replay()
            main.wait_stream(sv)
            torch.cuda.synchronize()
            for li, o in enumerate(outs):
                d = bits(o) != ref
                if bool(d.any()):
                    bad += 1
                    launches[li] = launches.get(li, 0) + 1
                    if VIC is None:
                        clips |= set(d.any(2).any(1).nonzero().flatten().tolist())
                        if os.environ.get("DETAIL") and shown < 6:
                            shown += 1
                            detail(o)
        print(f"aggressor {label} ({', '.join(c[0] for c in sel[:6])}{' ...' if len(sel) > 6 else ''}): "
              f"{bad}/{REPS * ROUNDS} STFT outputs differ, clips {sorted(clips)}, victim launches {launches}",
              flush=True)
        del ga
