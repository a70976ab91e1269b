"""bf16 model path (BASELINE config C3: `model.to(torch.bfloat16)`), on an MI355X.

Golden fixture: tests/golden/bf16_fwd.npz (tests/golden/gen_goldens.py::gen_bf16): the real
reference run as a bf16 model on the CPU (every op rounds to bf16).  The HIP path keeps bf16
weights and bf16 MFMA operands but accumulates in fp32 and keeps activations fp32 between
kernels, so it sits between the reference's bf16 and fp32 outputs.

Tolerances (SURVEY §8d for bf16): logits max-abs <= 0.1; per-frame argmax agreement >= 95 %
and token edit rate of the greedy lists <= 5 % against both the reference bf16 golden and the
fp32 golden (the reference's own bf16-vs-fp32 drift: max 0.030, argmax agreement 98.0 %, edit
rate 2.2-2.5 % on the bench batches).  The bench-shape batches (32 x 10 s per rank, C3) are in
tests/test_bench_workloads.py.
GEMM kernel: fp32 accumulation of exact bf16 products, vs float64 of the same rounded
operands: max-abs <= 2e-5 * scale.
"""

import json

import numpy as np
import pytest
import torch

from conftest import golden, golden_json, record_metric, token_edit_rate
from oracle import velocity_ref as R
from velocity_asr import synthetic as S

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def va():
    import velocity_asr
    from velocity_asr import _lib
    _lib.require_device()
    _lib.load()
    return velocity_asr


@pytest.fixture(scope="module")
def model_bf16(va):
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    return m.to(DEV).to(torch.bfloat16).eval()


@pytest.mark.parametrize("M,N,K", [(1, 64, 32), (257, 768, 192), (300, 512, 384), (130, 1000, 192), (5, 96, 240)])
@pytest.mark.parametrize("epi", ["none", "gelu", "residual"])
def test_gemm_bf16(va, M, N, K, epi):
    from velocity_asr import _lib, ops
    g = torch.Generator().manual_seed(M * 3 + N)
    a = torch.randn(M, K, generator=g)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, generator=g) * 0.1
    res = torch.randn(M, N, generator=g)
    ref = a.to(torch.bfloat16).double() @ w.double().T + b.double()
    e = {"none": _lib.EPI_NONE, "gelu": _lib.EPI_GELU, "residual": _lib.EPI_RESIDUAL}[epi]
    if epi == "gelu":
        ref = torch.nn.functional.gelu(ref)
    if epi == "residual":
        ref = ref + res.double()
    got = ops.gemm(a.to(DEV), w.to(DEV), b.to(DEV), epilogue=e,
                   aux=res.to(DEV) if epi == "residual" else None).cpu().double()
    scale = float(ref.abs().max()) + 1.0
    assert float((got - ref).abs().max()) <= 2e-5 * scale


def _check(logits, tokens_ref, greedy_ref, gold_logits=None, sub=1):
    agree = float((logits.argmax(-1) == tokens_ref).mean())
    rate = token_edit_rate(R.ctc_greedy_decode(logits), greedy_ref)
    record_metric("bf16_small", argmax_agreement=agree, token_edit_rate=rate)
    assert agree >= 0.95, f"argmax agreement {agree:.4f}"
    assert rate <= 0.05, f"token edit rate {rate:.4f}"
    d = None
    if gold_logits is not None:
        d = float(np.abs(logits[:, ::sub] - gold_logits).max())
        assert d <= 0.1, f"max |dlogit| {d:.4f}"
    return agree, d


@pytest.mark.parametrize("case,B,S_,seed", [("b2_3s", 2, 48000, 21), ("b2_10s", 2, 160000, 1234)])
def test_bf16_forward_vs_reference(va, model_bf16, case, B, S_, seed):
    z = golden("bf16_fwd.npz")
    audio = torch.from_numpy(S.make_audio(B, S_, seed=seed)).to(DEV)
    logits = model_bf16(va.compute_mel_spectrogram(audio)).cpu().numpy()
    greedy = json.loads(str(z[case + "__greedy"]))
    if case + "__logits" in z.files:
        agree, d = _check(logits, z[case + "__tokens"], greedy, z[case + "__logits"])
    else:
        agree, d = _check(logits, z[case + "__tokens"], greedy, z[case + "__logits_sub10"], sub=10)
    print(f"bf16 vs reference bf16 ({case}): argmax agreement {agree:.4f}, max |d| {d:.4f}")
    # and against the fp32 reference
    f = golden("fwd_b2_3s.npz" if case == "b2_3s" else "fwd_b2_10s.npz")
    agree32, _ = _check(logits, f["tokens"], golden_json("decode_fwd.json")["results"][case])
    print(f"bf16 vs reference fp32 ({case}): argmax agreement {agree32:.4f}")


def test_bf16_graphed_transcriber(va, model_bf16):
    from velocity_asr.pipeline import GraphedTranscriber, audio_to_token_ids, token_lists
    audio = torch.from_numpy(S.make_audio(4, 32000, seed=5)).to(DEV)
    te, le = audio_to_token_ids(model_bf16, audio)
    gt = GraphedTranscriber(model_bf16, 4, 32000)
    gt.audio.copy_(audio)
    gt.step()
    torch.cuda.synchronize()
    assert token_lists(gt.tokens, gt.lengths) == token_lists(te, le)


def test_composed_projection_bf16(va, monkeypatch):
    """The bf16 model's composed projection ([W_in; W_xdt W_in,x] as one bf16 GEMM, the default) vs the
    two GEMMs (VASR_BF16_COMPOSE=0): x and z are the same GEMM columns (bitwise), B | C | dt differ by
    one bf16 rounding of the composed weight instead of one of x_p (bf16 tolerance)."""
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    ssm = m.to(DEV).to(torch.bfloat16).eval().local_ssm.layers[3].ssm
    u = torch.from_numpy(np.random.default_rng(11).standard_normal((600, 192)).astype(np.float32)).to(DEV)
    monkeypatch.setenv("VASR_BF16_COMPOSE", "1")
    xz1, xdt1 = ssm.project(u)
    monkeypatch.setenv("VASR_BF16_COMPOSE", "0")
    xz0, xdt0 = ssm.project(u)
    assert torch.equal(xz1, xz0)
    err = (xdt1 - xdt0).abs().max().item()
    scale = xdt0.abs().max().item()
    assert err <= 2e-2 * scale, (err, scale)
