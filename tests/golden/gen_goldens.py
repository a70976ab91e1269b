#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REAL reference.

Container-only tool (the reference tree does not exist on the GPU box).  Run as

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference \
        python tests/golden/gen_goldens.py

It imports the reference ``velocity_asr`` package read-only, loads the portable
weight recipe (``velocity-asr_amd/velocity_asr/synthetic.py``) by file path, runs
the reference CPU path on seeded inputs and writes small .npz/.json fixtures
(inputs are regenerated from the recorded seeds; only outputs and small inputs
are stored).  Every file records the torch version, thread count and batch
shape, because the reference CPU path is not batch-invariant at the 1e-6 level
("Batch-invariance").
"""

import importlib.util
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
SYN_PATH = os.path.join(REPO, "velocity-asr_amd", "velocity_asr", "synthetic.py")

spec = importlib.util.spec_from_file_location("vasr_synthetic", SYN_PATH)
syn = importlib.util.module_from_spec(spec)
spec.loader.exec_module(syn)

import velocity_asr as ref  # noqa: E402  (the reference, via PYTHONPATH)
from velocity_asr import audio as ref_audio  # noqa: E402
from velocity_asr import decode as ref_decode  # noqa: E402
from velocity_asr import training as ref_training  # noqa: E402
from velocity_asr.ssm import SelectiveSSM  # noqa: E402

assert os.path.realpath(os.path.dirname(ref.__file__)).startswith("/root/reference"), ref.__file__

torch.set_num_threads(8)
META = dict(torch=torch.__version__, threads=torch.get_num_threads(), numpy=np.__version__)


def build_model(config=None, seed=0):
    cfg = ref.VelocityASRConfig(**(config or {}))
    model = ref.VELOCITYASR(cfg)
    weights = syn.make_weights(config, seed=seed)
    sd = model.state_dict()
    assert list(sd.keys()) == list(weights.keys()), "recipe key order != reference state_dict"
    for k, v in sd.items():
        assert tuple(v.shape) == weights[k].shape, (k, v.shape, weights[k].shape)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in weights.items()}, strict=True)
    model.eval()
    return model


def meta(**kw):
    d = dict(META)
    d.update(kw)
    return np.array(json.dumps(d))


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {name}: {os.path.getsize(path)/1024:.1f} KiB")


# --------------------------------------------------------------------------- mel
def gen_mel():
    out = {}
    cases = {
        "rand_b2_1s": syn.make_audio(2, 16000, seed=11),
        "rand_b2_10s": syn.make_audio(2, 160000, seed=1234),
        "chirp_3s": syn.make_chirp(48000)[None],
        "zero_1s": np.zeros((1, 16000), np.float32),
        "short_201": syn.make_audio(1, 201, seed=5),
        "short_400": syn.make_audio(1, 400, seed=6),
        "odd_16333": syn.make_audio(3, 16333, seed=8),
    }
    for name, audio in cases.items():
        with torch.no_grad():
            mel = ref_audio.compute_mel_spectrogram(torch.from_numpy(audio))
        out[name] = mel.numpy()
        if name in ("chirp_3s", "zero_1s", "short_201", "short_400"):
            out[name + "__audio"] = audio
    # 1-D input squeezes (audio.py:89-91, 140-141)
    a1 = syn.make_audio(1, 8000, seed=9)[0]
    out["oned_8000"] = ref_audio.compute_mel_spectrogram(torch.from_numpy(a1)).numpy()
    fb = ref_audio._create_mel_filterbank(400, 80, 16000, torch.device("cpu"))
    out["filterbank"] = fb.numpy()
    out["hann"] = torch.hann_window(400).numpy()
    out["meta"] = meta(seeds=dict(rand_b2_1s=11, rand_b2_10s=1234, short_201=5, short_400=6,
                                  odd_16333=8, oned_8000=9, chirp=7))
    save("mel.npz", **out)


# --------------------------------------------------------------------------- scan
def scan_inputs(seed, B, L, Di, N):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((B, L, Di)).astype(np.float32)
    dt = np.log1p(np.exp(rng.standard_normal((B, L, Di)) * 0.7 - 1.0)).astype(np.float32)
    Bm = rng.standard_normal((B, L, N)).astype(np.float32)
    Cm = rng.standard_normal((B, L, N)).astype(np.float32)
    A_log = (np.log(np.arange(1, N + 1)) + 0.01 * rng.standard_normal(N)).astype(np.float32)
    D = (1.0 + 0.1 * rng.standard_normal(Di)).astype(np.float32)
    return x, dt, Bm, Cm, A_log, D


SCAN_CASES = [
    # (name, seed, B, L, Di, N)
    ("L1", 100, 2, 1, 8, 64),
    ("L2", 101, 2, 2, 8, 64),
    ("L3", 102, 2, 3, 8, 64),
    ("L7", 103, 1, 7, 16, 64),
    ("L16", 104, 1, 16, 8, 64),
    ("L17", 105, 1, 17, 8, 64),
    ("L64_N32", 106, 2, 64, 16, 32),
    ("L100", 107, 1, 100, 8, 64),
    ("L187_N32", 108, 1, 187, 8, 32),
    ("L501", 109, 2, 501, 8, 64),
    ("L1501", 110, 1, 1501, 4, 64),
]


def gen_scan():
    out = {}
    for name, seed, B, L, Di, N in SCAN_CASES:
        x, dt, Bm, Cm, A_log, D = scan_inputs(seed, B, L, Di, N)
        ssm = SelectiveSSM(d_model=Di // 2, state_dim=N, expand_ratio=2)
        with torch.no_grad():
            ssm.D.copy_(torch.from_numpy(D))
            A = -torch.exp(torch.from_numpy(A_log))
            tx, tdt, tB, tC = (torch.from_numpy(v) for v in (x, dt, Bm, Cm))
            yp = ssm._parallel_scan(tx, tdt, A, tB, tC)
            ys = ssm._sequential_scan(tx, tdt, A, tB, tC)
        out[name + "__parallel"] = yp.numpy()
        out[name + "__sequential"] = ys.numpy()
    out["meta"] = meta(cases=[list(c) for c in SCAN_CASES],
                       inputs="tests/golden/gen_goldens.py:scan_inputs(seed,B,L,Di,N)")
    save("scan.npz", **out)


# --------------------------------------------------------------------------- forward
def topk_pack(prefix, logits, out, every=25):
    lg = torch.from_numpy(logits) if isinstance(logits, np.ndarray) else logits
    vals, idx = torch.topk(lg, 5, dim=-1)
    out[prefix + "tokens"] = lg.argmax(-1).numpy().astype(np.int32)
    out[prefix + "top5_val"] = vals.numpy()
    out[prefix + "top5_idx"] = idx.numpy().astype(np.int32)
    out[prefix + "frames"] = np.arange(0, lg.shape[1], every, dtype=np.int32)
    out[prefix + "logits_sub"] = lg[:, ::every].numpy()
    out[prefix + "margin_min"] = np.array((vals[..., 0] - vals[..., 1]).min().item(), np.float32)
    out[prefix + "abs_sum"] = lg.abs().sum(dim=(1, 2)).double().numpy()


def run_forward(model, audio):
    with torch.no_grad():
        mel = ref_audio.compute_mel_spectrogram(torch.from_numpy(audio))
        logits, feats = model(mel, return_features=True)
    return mel, logits, feats


def greedy_json(logits):
    return ref_decode.ctc_greedy_decode(logits)


def gen_forward():
    model = build_model()
    decoded = {}

    # (i) per-stage features at B=2 x 3 s
    audio = syn.make_audio(2, 48000, seed=21)
    mel, logits, feats = run_forward(model, audio)
    save("fwd_b2_3s.npz", mel=mel.numpy(), temporal_binding=feats["temporal_binding"].numpy(),
         local_features=feats["local_features"].numpy(),
         fused_features=feats["fused_features"].numpy(), logits=logits.numpy(),
         tokens=logits.argmax(-1).numpy().astype(np.int32),
         meta=meta(audio="make_audio(2, 48000, seed=21)", weights="make_weights(None, seed=0)",
                   batch=[2, 48000]))
    decoded["b2_3s"] = greedy_json(logits)
    decoded["b2_3s_ts"] = ref_decode.ctc_greedy_decode_with_timestamps(logits)

    # (ii) headline shape, two utterances of 10 s
    audio = syn.make_audio(2, 160000, seed=1234)
    mel, logits, feats = run_forward(model, audio)
    out = {}
    topk_pack("", logits, out)
    out["local_sub"] = feats["local_features"][:, ::25].numpy()
    out["meta"] = meta(audio="make_audio(2, 160000, seed=1234)", weights="make_weights(None, seed=0)",
                       batch=[2, 160000])
    save("fwd_b2_10s.npz", **out)
    decoded["b2_10s"] = greedy_json(logits)

    # (iii) long utterance, 30 s (L=1501, P=2048, K1=187, K2=46)
    audio = syn.make_audio(1, 480000, seed=4321)
    mel, logits, feats = run_forward(model, audio)
    out = {}
    topk_pack("", logits, out, every=50)
    out["meta"] = meta(audio="make_audio(1, 480000, seed=4321)", weights="make_weights(None, seed=0)",
                       batch=[1, 480000])
    save("fwd_b1_30s.npz", **out)
    decoded["b1_30s"] = greedy_json(logits)

    # (iv) chirp 'speech-like' clip, B=1 x 3 s
    audio = syn.make_chirp(48000)[None]
    mel, logits, feats = run_forward(model, audio)
    save("fwd_chirp_3s.npz", logits=logits.numpy(), tokens=logits.argmax(-1).numpy().astype(np.int32),
         meta=meta(audio="make_chirp(48000)[None]", batch=[1, 48000]))
    decoded["chirp_3s"] = greedy_json(logits)

    # (v) edge lengths: L = 1, 2, 6, 26, 51; pool sizes clamp to L
    edge = {}
    for S, seed in ((201, 31), (400, 32), (1600, 33), (8000, 34), (16333, 35)):
        audio = syn.make_audio(1, S, seed=seed)
        mel, logits, feats = run_forward(model, audio)
        edge[f"S{S}__logits"] = logits.numpy()
        edge[f"S{S}__tokens"] = logits.argmax(-1).numpy().astype(np.int32)
    edge["meta"] = meta(audio="make_audio(1, S, seed) for (S, seed) in (201,31),(400,32),(1600,33),(8000,34),(16333,35)")
    save("fwd_edge.npz", **edge)

    # (vi) raw-mel input (model API takes mel, not audio): randn mel like test_vel.py
    rng = np.random.default_rng(41)
    mel_in = rng.standard_normal((2, 500, 80)).astype(np.float32)
    with torch.no_grad():
        logits = model(torch.from_numpy(mel_in))
    save("fwd_melin_500.npz", logits=logits.numpy(), tokens=logits.argmax(-1).numpy().astype(np.int32),
         meta=meta(mel="default_rng(41).standard_normal((2,500,80))", batch=[2, 500]))

    with open(os.path.join(HERE, "decode_fwd.json"), "w") as f:
        json.dump({"meta": json.loads(str(meta())), "results": decoded}, f)
    print("wrote decode_fwd.json")


def gen_forward_sequential():
    cfg = dict(scan_mode="sequential")
    model = build_model(cfg)
    audio = syn.make_audio(2, 48000, seed=21)
    mel, logits, feats = run_forward(model, audio)
    save("fwd_seq_b2_3s.npz", logits=logits.numpy(), local_features=feats["local_features"].numpy(),
         tokens=logits.argmax(-1).numpy().astype(np.int32),
         meta=meta(config=cfg, audio="make_audio(2, 48000, seed=21)", batch=[2, 48000]))


SMALL_CFG = dict(d_model=96, ssm_layers=2, ssm_state_dim=32, global_ssm_state_dim=16,
                 attention_heads=2, attention_dim=24, vocab_size=50)


def gen_forward_small_config():
    model = build_model(SMALL_CFG, seed=3)
    audio = syn.make_audio(2, 32000, seed=51)
    mel, logits, feats = run_forward(model, audio)
    save("fwd_smallcfg.npz", logits=logits.numpy(), tokens=logits.argmax(-1).numpy().astype(np.int32),
         local_features=feats["local_features"].numpy(),
         meta=meta(config=SMALL_CFG, weights_seed=3, audio="make_audio(2, 32000, seed=51)",
                   batch=[2, 32000]))


# --------------------------------------------------------------------------- decode / wer
def gen_decode():
    rng = np.random.default_rng(61)
    cases = {}
    # sticky random token streams with blanks and repeats, V=12
    for i, (B, L, V) in enumerate(((3, 40, 12), (2, 1, 5), (1, 64, 3), (2, 33, 1000))):
        toks = np.zeros((B, L), np.int64)
        for b in range(B):
            cur = 0
            for t in range(L):
                r = rng.random()
                if r < 0.3:
                    cur = 0
                elif r < 0.6:
                    cur = int(rng.integers(0, V))
                toks[b, t] = cur
        logits = rng.standard_normal((B, L, V)).astype(np.float32)
        # make the chosen token the argmax
        logits[np.arange(B)[:, None], np.arange(L)[None], toks] = 10.0
        lt = torch.from_numpy(logits)
        cases[f"c{i}"] = dict(
            logits=logits.tolist(),
            greedy=ref_decode.ctc_greedy_decode(lt),
            greedy_nocollapse=ref_decode.ctc_greedy_decode(lt, collapse_repeated=False),
            timestamps=[[list(tk), [list(s) for s in ts]] for tk, ts in
                        ref_decode.ctc_greedy_decode_with_timestamps(lt)],
        )
    vocab = ref_decode.create_default_vocabulary(1000)
    dec = ref_decode.CTCDecoder(vocab)
    texts = dec.decode_greedy(torch.from_numpy(np.array(cases["c3"]["logits"], np.float32)))
    wer_cases = [
        (["the cat sat", "hello world"], ["the cat sat on", "hello word"]),
        ([""], ["a b c"]),
        (["A B"], ["a b"]),
        (["x y z"], [""]),
    ]
    wer = [dict(pred=p, ref=r, wer=ref_training.compute_wer(p, r), cer=ref_training.compute_cer(p, r))
           for p, r in wer_cases]
    out = dict(meta=json.loads(str(meta())), cases=cases, vocab_head=vocab[:80], vocab_len=len(vocab),
               vocab_tail=vocab[-3:], texts_c3=texts, wer=wer,
               vocab_small=ref_decode.create_default_vocabulary(10))
    with open(os.path.join(HERE, "decode.json"), "w") as f:
        json.dump(out, f)
    print("wrote decode.json")


# --------------------------------------------------------------------------- int8 (C5)
QAT_MAP_RE = (".linear.", ".conv.")


def qat_state_from_fp32(qmodel, sd):
    """The reference's prepare_model_for_qat re-initialises the replaced modules
    (quantize.py:295-313, SURVEY a17 defect i); carry the fp32 weights over instead:
    `X.linear.weight` / `X.conv.weight` take `X.weight`, quantizer buffers keep their init."""
    out = {}
    for k, v in qmodel.state_dict().items():
        if k in sd:
            out[k] = sd[k]
            continue
        for seg in QAT_MAP_RE:
            head, _, tail = k.rpartition(seg)
            if head and (head + "." + tail) in sd:
                out[k] = sd[head + "." + tail]
                break
        else:
            out[k] = v
    return out


def qat_model(calib_audio):
    """fp32 weights in the reference's QAT modules, calibrated with the intended semantics:
    weight quantizers on their weights, activation quantizers on the outputs of one
    calibration forward (weights fake-quantized, activations still pass-through)."""
    from velocity_asr.quantize import FakeQuantize, QuantizedConv1d, QuantizedLinear, prepare_model_for_qat
    model = build_model()
    sd = model.state_dict()
    qmodel = prepare_model_for_qat(model)
    qmodel.load_state_dict(qat_state_from_fp32(qmodel, sd), strict=True)
    qmodel.eval()
    qmods = {n: m for n, m in qmodel.named_modules() if isinstance(m, (QuantizedLinear, QuantizedConv1d))}
    with torch.no_grad():
        for n, m in qmods.items():
            inner = m.linear if isinstance(m, QuantizedLinear) else m.conv
            m.weight_quantizer.calibrate(inner.weight)
        seen = {}
        hooks = [m.register_forward_hook(lambda mod, inp, out, n=n: seen.__setitem__(n, out.detach().clone()))
                 for n, m in qmods.items()]
        mel = ref_audio.compute_mel_spectrogram(torch.from_numpy(calib_audio))
        qmodel(mel)
        for h in hooks:
            h.remove()
        for n, m in qmods.items():
            m.activation_quantizer.calibrate(seen[n])
    return qmodel, sorted(qmods)


def gen_int8():
    calib = syn.make_audio(2, 48000, seed=71)
    qmodel, names = qat_model(calib)
    out = {}
    for k, v in qmodel.state_dict().items():
        if "quantizer" in k:
            out["q__" + k] = v.numpy()
    audio = syn.make_audio(2, 48000, seed=21)
    mel, logits, feats = run_forward(qmodel, audio)
    out["logits"] = logits.numpy()
    out["tokens"] = logits.argmax(-1).numpy().astype(np.int32)
    out["temporal_binding"] = feats["temporal_binding"].numpy()
    out["fused_features"] = feats["fused_features"].numpy()
    out["greedy"] = np.array(json.dumps(ref_decode.ctc_greedy_decode(logits)))
    # the reference's own calibrate_model (quantize.py:325-369) on fresh QAT modules: eval-mode
    # forwards pass through, then every quantizer is marked calibrated with scale 1, zp 0
    from velocity_asr.quantize import calibrate_model, prepare_model_for_qat
    torch.manual_seed(0)
    m2 = prepare_model_for_qat(build_model())
    sd2 = qat_state_from_fp32(m2, build_model().state_dict())
    m2.load_state_dict(sd2, strict=True)
    calibrate_model(m2, [(torch.from_numpy(np.zeros((1, 100, 80), np.float32)),)], num_batches=1, device="cpu")
    with torch.no_grad():
        lg2 = m2(mel)
    out["refcal_logits"] = lg2.numpy()
    out["modules"] = np.array(json.dumps(names))
    # element-level known answers of FakeQuantize itself (bit-exact pins for the kernels)
    from velocity_asr.quantize import FakeQuantize
    rng = np.random.default_rng(72)
    x = (rng.standard_normal((48, 40)) * 2.0).astype(np.float32)
    x[0, :8] = [0.0, -0.0, 1e-12, -1e-12, 3.4e38, -3.4e38, 0.5, -0.5]
    fq_cases = [("asym8", dict(bits=8, symmetric=False, per_channel=False)),
                ("sym8_pc", dict(bits=8, symmetric=True, per_channel=True, channel_dim=0)),
                ("sym8", dict(bits=8, symmetric=True, per_channel=False)),
                ("asym4", dict(bits=4, symmetric=False, per_channel=False)),
                ("sym6_pc", dict(bits=6, symmetric=True, per_channel=True, channel_dim=0))]
    for name, kw in fq_cases:
        fq = FakeQuantize(**kw).eval()
        with torch.no_grad():
            # per-tensor: calibrate on rows 1.. (row 0 holds extremes that then clamp)
            fq.calibrate(torch.from_numpy(x if kw["per_channel"] else x[1:]))
            y = fq(torch.from_numpy(x))
        out[f"fq_{name}__y"] = y.numpy()
        out[f"fq_{name}__scale"] = fq.scale.numpy()
        out[f"fq_{name}__zp"] = fq.zero_point.numpy()
    out["fq_x"] = x
    out["fq_cases"] = np.array(json.dumps(fq_cases))
    out["meta"] = meta(calib="make_audio(2, 48000, seed=71)", audio="make_audio(2, 48000, seed=21)",
                       weights="make_weights(None, seed=0) carried into prepare_model_for_qat modules",
                       batch=[2, 48000])
    save("int8_b2_3s.npz", **out)


# --------------------------------------------------------------------------- beam search
def gen_beam():
    """ctc_beam_search (decode.py:128-217) on the decode.json logit cases and on soft random
    logits (many competing prefixes), beam widths 1, 3, 5, 10."""
    rng = np.random.default_rng(81)
    dec = json.load(open(os.path.join(HERE, "decode.json")))
    cases = {k: np.array(v["logits"], np.float32) for k, v in dec["cases"].items()}
    cases["soft_v6"] = (rng.standard_normal((2, 30, 6)) * 1.5).astype(np.float32)
    cases["soft_v40"] = (rng.standard_normal((2, 25, 40)) * 2.0).astype(np.float32)
    cases["soft_l0"] = np.zeros((1, 0, 5), np.float32)
    out = {"meta": json.loads(str(meta())), "cases": {}}
    for name, lg in cases.items():
        res = {}
        for w in (1, 3, 5, 10):
            r = ref_decode.ctc_beam_search(torch.from_numpy(lg), beam_width=w)
            res[str(w)] = [[[list(map(int, d.tokens)), float(d.score)] for d in beams] for beams in r]
        out["cases"][name] = {"logits": lg.tolist() if name.startswith("soft") else None, "beams": res}
    with open(os.path.join(HERE, "beam.json"), "w") as f:
        json.dump(out, f)
    print("wrote beam.json")


# --------------------------------------------------------------------------- bf16 (C3)
def gen_bf16():
    """The reference run as a bf16 model: model.to(torch.bfloat16), fp32 audio -> mel, mel cast
    to bf16 (every op of the forward then computes in bf16 on the CPU)."""
    model = build_model().to(torch.bfloat16)
    out = {}
    for name, (B, S, seed) in {"b2_3s": (2, 48000, 21), "b2_10s": (2, 160000, 1234)}.items():
        audio = syn.make_audio(B, S, seed=seed)
        with torch.no_grad():
            mel = ref_audio.compute_mel_spectrogram(torch.from_numpy(audio))
            logits = model(mel.to(torch.bfloat16)).float()
        out[name + ("__logits" if S < 100000 else "__logits_sub10")] = (logits.numpy() if S < 100000
                                                                          else logits[:, ::10].numpy())
        out[name + "__tokens"] = logits.argmax(-1).numpy().astype(np.int32)
        out[name + "__greedy"] = np.array(json.dumps(ref_decode.ctc_greedy_decode(logits)))
    out["meta"] = meta(weights="make_weights(None, seed=0) -> model.to(bfloat16)",
                       audio="b2_3s: make_audio(2, 48000, seed=21); b2_10s: make_audio(2, 160000, seed=1234)")
    save("bf16_fwd.npz", **out)


# --------------------------------------------------------------------------- full bench batches
def _tokens_pack(prefix, model, audio, chunk, out, decoded):
    """Reference forward over `audio` in chunks of `chunk` clips (the reference CPU path needs
    ~0.5 GB per 10-s clip); argmax tokens, top-2 margin per frame, greedy lists."""
    toks, margins, greedy = [], [], []
    for i in range(0, audio.shape[0], chunk):
        with torch.no_grad():
            mel = ref_audio.compute_mel_spectrogram(torch.from_numpy(audio[i:i + chunk]))
            logits = model(mel)
        top2 = torch.topk(logits, 2, dim=-1)
        toks.append(logits.argmax(-1).numpy().astype(np.int16))
        margins.append((top2.values[..., 0] - top2.values[..., 1]).numpy().astype(np.float32))
        greedy.extend(ref_decode.ctc_greedy_decode(logits))
        print(f"  {prefix}: clips {i}..{i + chunk - 1} done", flush=True)
    out[prefix + "tokens"] = np.concatenate(toks)
    out[prefix + "margin"] = np.concatenate(margins)
    decoded[prefix.rstrip("_")] = greedy


def gen_fullbatch():
    """Every clip of the bench workloads pinned to the reference:
    C2 = make_audio(32, 160000, seed=1234) (bench.py rank 0), all 32 clips, chunks of 8;
    C4 = make_audio(32, 480000, seed=1234), the first 8 clips, chunks of 2."""
    model = build_model()
    out, decoded = {}, {}
    _tokens_pack("c2_", model, syn.make_audio(32, 160000, seed=1234), 8, out, decoded)
    _tokens_pack("c4_", model, syn.make_audio(32, 480000, seed=1234)[:8], 2, out, decoded)
    out["greedy"] = np.array(json.dumps(decoded))
    out["meta"] = meta(c2="make_audio(32, 160000, seed=1234), reference run in chunks of 8",
                       c4="make_audio(32, 480000, seed=1234)[:8], reference run in chunks of 2",
                       weights="make_weights(None, seed=0)")
    save("fwd_fullbatch.npz", **out)


def gen_c4full():
    """All 32 clips of C4 = make_audio(32, 480000, seed=1234), written into
    fwd_fullbatch.npz in place of the first-8 entries (c2 kept); the reference in chunks of 4.
    The first 8 clips' greedy lists must equal the earlier chunks-of-2 run (batch invariance)."""
    path = os.path.join(HERE, "fwd_fullbatch.npz")
    old = np.load(path, allow_pickle=False)
    out = {k: old[k] for k in old.files if k not in ("greedy", "meta")}
    decoded = json.loads(str(old["greedy"]))
    prev = decoded.get("c4")
    model = build_model()
    _tokens_pack("c4_", model, syn.make_audio(32, 480000, seed=1234), 4, out, decoded)
    if prev is not None and decoded["c4"][:len(prev)] != prev:
        raise AssertionError("C4: the first clips' reference tokens changed with the chunking")
    out["greedy"] = np.array(json.dumps(decoded))
    out["meta"] = meta(c2="make_audio(32, 160000, seed=1234), reference run in chunks of 8",
                       c4="make_audio(32, 480000, seed=1234), all 32 clips, reference run in chunks of 4",
                       weights="make_weights(None, seed=0)")
    save("fwd_fullbatch.npz", **out)


TIE_MARGIN = 2e-5  # near-ties: reference top-2 margins below this (> 2x the largest |dlogit| measured)


def _logits_pack(prefix, model, audio, chunk, every, out, check_tokens=None):
    """Reference logits at the headline shapes: frames 0::every of every
    clip (all 1000 classes), plus the full rows of every near-tie frame (reference top-2 margin
    < TIE_MARGIN) with their (clip, frame) indices; the argmax tokens must equal the earlier
    tokens-only golden of the same chunking."""
    subs, ties_idx, ties_rows, toks = [], [], [], []
    for i in range(0, audio.shape[0], chunk):
        with torch.no_grad():
            mel = ref_audio.compute_mel_spectrogram(torch.from_numpy(audio[i:i + chunk]))
            logits = model(mel)
        subs.append(logits[:, ::every].numpy())
        top2 = torch.topk(logits, 2, dim=-1).values
        m = (top2[..., 0] - top2[..., 1]).numpy()
        for b, f in np.argwhere(m < TIE_MARGIN):
            ties_idx.append((i + int(b), int(f)))
            ties_rows.append(logits[b, f].numpy())
        toks.append(logits.argmax(-1).numpy().astype(np.int16))
        print(f"  {prefix}: clips {i}..{i + chunk - 1} done", flush=True)
    toks = np.concatenate(toks)
    if check_tokens is not None and not np.array_equal(toks, check_tokens):
        raise AssertionError(f"{prefix}: argmax tokens differ from the tokens-only golden")
    out[prefix + "every"] = np.array(every, np.int32)
    out[prefix + "logits_sub"] = np.concatenate(subs).astype(np.float32)
    out[prefix + "tie_idx"] = np.array(ties_idx, np.int32).reshape(-1, 2)
    out[prefix + "tie_logits"] = np.array(ties_rows, np.float32).reshape(-1, out[prefix + "logits_sub"].shape[-1])


def gen_headline_logits():
    """fwd_headline_logits.npz: logits for all 32 clips of C2 (32 x 10 s, frames 0::25, reference
    in chunks of 8) and C4 (32 x 30 s, frames 0::75, chunks of 4) -- the same chunkings as
    fwd_fullbatch.npz, whose tokens they must reproduce -- and every near-tie frame's full row."""
    model = build_model()
    full = np.load(os.path.join(HERE, "fwd_fullbatch.npz"), allow_pickle=False)
    out = {}
    _logits_pack("c2_", model, syn.make_audio(32, 160000, seed=1234), 8, 25, out, full["c2_tokens"])
    _logits_pack("c4_", model, syn.make_audio(32, 480000, seed=1234), 4, 75, out, full["c4_tokens"])
    out["meta"] = meta(c2="make_audio(32, 160000, seed=1234), reference run in chunks of 8, frames 0::25",
                       c4="make_audio(32, 480000, seed=1234), reference run in chunks of 4, frames 0::75",
                       tie_margin=TIE_MARGIN, weights="make_weights(None, seed=0)")
    save("fwd_headline_logits.npz", **out)


def _greedy_pack(prefix, model, audio, chunk, out, decoded, cast=None):
    """Like _tokens_pack for a model whose forward takes `cast(mel)` (bf16): argmax tokens and
    greedy lists only (margins are meaningless for the statistical configs)."""
    toks, greedy = [], []
    for i in range(0, audio.shape[0], chunk):
        with torch.no_grad():
            mel = ref_audio.compute_mel_spectrogram(torch.from_numpy(audio[i:i + chunk]))
            logits = model(cast(mel) if cast else mel).float()
        toks.append(logits.argmax(-1).numpy().astype(np.int16))
        greedy.extend(ref_decode.ctc_greedy_decode(logits))
        print(f"  {prefix}: clips {i}..{i + chunk - 1} done", flush=True)
    out[prefix + "tokens"] = np.concatenate(toks)
    decoded[prefix.rstrip("_")] = greedy


def gen_benchsets():
    """The bench's per-rank workloads for every BASELINE config:
    rank r of `bench.py --gpus N` transcribes make_audio(32, 160000, seed=1234 + r).
      fp32 (C2 at N > 1): ranks 1..7 (rank 0 is fwd_fullbatch.npz's c2), chunks of 8;
      bf16 (C3 = 256 clips over 8 ranks): ranks 0..7 with model.to(bfloat16), chunks of 8;
      int8 (C5): rank 0 with the intended-semantics QAT model calibrated as bench.py does
      (make_audio(2, 48000, seed=71)).
    Chunked runs: the reference CPU path is batch-invariant to ~2e-6 (SURVEY §8 e)."""
    which = os.environ.get("VASR_BENCHSETS", "fp32,bf16,int8").split(",")
    path = os.path.join(HERE, "fwd_benchsets.npz")
    out, decoded = {}, {}
    if os.path.exists(path):  # incremental: keep what an earlier run wrote
        old = np.load(path, allow_pickle=False)
        out = {k: old[k] for k in old.files if k not in ("greedy", "meta")}
        decoded = json.loads(str(old["greedy"]))
    if "fp32" in which:
        model = build_model()
        for r in range(1, 8):
            _tokens_pack(f"fp32_r{r}_", model, syn.make_audio(32, 160000, seed=1234 + r), 8, out, decoded)
    if "bf16" in which:
        model = build_model().to(torch.bfloat16)
        for r in range(8):
            _greedy_pack(f"bf16_r{r}_", model, syn.make_audio(32, 160000, seed=1234 + r), 8, out, decoded,
                         cast=lambda m: m.to(torch.bfloat16))
    if "int8" in which:
        qmodel, _ = qat_model(syn.make_audio(2, 48000, seed=71))
        _greedy_pack("int8_r0_", qmodel, syn.make_audio(32, 160000, seed=1234), 8, out, decoded)
    out["greedy"] = np.array(json.dumps(decoded))
    out["meta"] = meta(audio="rank r: make_audio(32, 160000, seed=1234 + r)", weights="make_weights(None, seed=0)",
                       fp32="ranks 1..7, chunks of 8", bf16="model.to(bfloat16), mel cast to bf16, ranks 0..7",
                       int8="gen_goldens.qat_model(make_audio(2, 48000, seed=71)), rank 0")
    save("fwd_benchsets.npz", **out)


STATEDIM_CFGS = {"sd8": dict(ssm_state_dim=8, global_ssm_state_dim=8),
                 "sd48": dict(ssm_state_dim=48, global_ssm_state_dim=24),
                 "sd128": dict(ssm_state_dim=128, global_ssm_state_dim=128)}
STATEDIM_SCANS = [("N8", 120, 2, 100, 16, 8), ("N48", 121, 1, 257, 16, 48), ("N128", 122, 2, 301, 8, 128)]


def gen_statedims():
    """State dims the scan kernels are not built for: SelectiveSSM(state_dim)
    and VelocityASRConfig.ssm_state_dim / global_ssm_state_dim take any N (ssm.py:32-90,
    model.py:23-68).  Whole-model forwards at N = 8, 48, 128 and scans at the same N."""
    out = {}
    for name, cfg in STATEDIM_CFGS.items():
        model = build_model(cfg, seed=5)
        audio = syn.make_audio(2, 32000, seed=52)
        mel, logits, feats = run_forward(model, audio)
        out[name + "__logits_sub4"] = logits[:, ::4].numpy()
        out[name + "__tokens"] = logits.argmax(-1).numpy().astype(np.int32)
    for name, seed, B, L, Di, N in STATEDIM_SCANS:
        x, dt, Bm, Cm, A_log, D = scan_inputs(seed, B, L, Di, N)
        ssm = SelectiveSSM(d_model=Di // 2, state_dim=N, expand_ratio=2)
        with torch.no_grad():
            ssm.D.copy_(torch.from_numpy(D))
            A = -torch.exp(torch.from_numpy(A_log))
            tx, tdt, tB, tC = (torch.from_numpy(v) for v in (x, dt, Bm, Cm))
            out[name + "__parallel"] = ssm._parallel_scan(tx, tdt, A, tB, tC).numpy()
            out[name + "__sequential"] = ssm._sequential_scan(tx, tdt, A, tB, tC).numpy()
    out["meta"] = meta(configs=STATEDIM_CFGS, weights_seed=5, audio="make_audio(2, 32000, seed=52)",
                       scans=[list(c) for c in STATEDIM_SCANS],
                       scan_inputs="tests/golden/gen_goldens.py:scan_inputs(seed,B,L,Di,N)")
    save("fwd_statedims.npz", **out)


# --------------------------------------------------------------------------- CLI output
CLI_CLIPS = {"clip_2s.wav": ("make_audio(1, 32000, seed=91)[0]", lambda: syn.make_audio(1, 32000, seed=91)[0]),
             "chirp_3s.wav": ("make_chirp(48000)", lambda: syn.make_chirp(48000)),
             "clip_10s.wav": ("make_audio(2, 160000, seed=1234)[1]", lambda: syn.make_audio(2, 160000, seed=1234)[1])}


def gen_cli():
    """The reference's own scripts/transcribe.py:transcribe_file (text and --timestamps JSON).
    Its load_audio needs torchaudio (absent), so the module's `load_audio` name is rebound to
    return the clip; everything after it (mel, forward, decode, word grouping) is the reference."""
    spec = importlib.util.spec_from_file_location("ref_transcribe_script", "/root/reference/scripts/transcribe.py")
    tr = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tr)
    model = build_model()
    decoder = ref_decode.CTCDecoder(ref_decode.create_default_vocabulary(1000))
    res = {}
    for name, (recipe, make) in CLI_CLIPS.items():
        clip = torch.from_numpy(make())
        tr.load_audio = lambda path, _c=clip: _c
        res[name] = {"recipe": recipe,
                     "text": tr.transcribe_file(model, name, decoder, "cpu", include_timestamps=False),
                     "timestamps": tr.transcribe_file(model, name, decoder, "cpu", include_timestamps=True)}
    with open(os.path.join(HERE, "cli_transcribe.json"), "w") as f:
        json.dump({"meta": json.loads(str(meta(weights="make_weights(None, seed=0)"))), "clips": res}, f, indent=1)
    print("wrote cli_transcribe.json")


if __name__ == "__main__":
    which = sys.argv[1:] or ["mel", "scan", "forward", "sequential", "small", "decode", "int8", "bf16", "beam",
                             "fullbatch", "cli", "statedims"]
    if "mel" in which:
        gen_mel()
    if "scan" in which:
        gen_scan()
    if "forward" in which:
        gen_forward()
    if "sequential" in which:
        gen_forward_sequential()
    if "small" in which:
        gen_forward_small_config()
    if "decode" in which:
        gen_decode()
    if "int8" in which:
        gen_int8()
    if "bf16" in which:
        gen_bf16()
    if "beam" in which:
        gen_beam()
    if "fullbatch" in which:
        gen_fullbatch()
    if "c4full" in which:  # ~4 min on 8 threads: not in the default list
        gen_c4full()
    if "headline" in which:  # ~3 min on 8 threads: not in the default list
        gen_headline_logits()
    if "benchsets" in which:  # long (~30 min on 8 threads): not in the default list
        gen_benchsets()
    if "statedims" in which:
        gen_statedims()
    if "cli" in which:
        gen_cli()
