"""Concurrent streams: results must not depend on what else runs on the chip.

Two utterance groups replayed as HIP graphs on concurrent streams (GraphedTranscriber(streams=2),
the two-group schedule of bench.py) must give every clip the reference's tokens on every replay
(tests/golden/fwd_fullbatch.npz, the reference CPU path on make_audio(32, 160000, seed=1234);
reference callers: scripts/transcribe.py:69-78, evaluate.py:91-98; forward model.py:333-368).
Before round 4 they did not: group 1's clips came back wrong in 0.5-8 % of replays
(profiles/r03ao, r04a).  The kernel-level form: a kernel's output run beside a co-resident kernel
of another stream equals its output alone, bit for bit (tools/diag/interference.py,
profiles/r04b-r04g)."""
import json

import pytest
import torch

from conftest import golden
from velocity_asr import synthetic as S

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def model():
    import velocity_asr as va
    from velocity_asr import _lib
    _lib.require_device()
    _lib.load()
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in S.make_weights(None, seed=0).items()}, strict=True)
    return m.to(DEV).eval()


def test_two_group_graphs_every_replay_matches_reference(model):
    """32 x 10 s clips as two 16-clip graphs replayed concurrently, 12 replays (the audio rewritten
    before each): every clip's token list equals the reference's in every replay."""
    from velocity_asr.pipeline import GraphedTranscriber, token_lists
    ref = json.loads(str(golden("fwd_fullbatch.npz")["greedy"]))["c2"]
    audio = torch.from_numpy(S.make_audio(32, 160000, seed=1234)).to(DEV)
    tr = GraphedTranscriber(model, 32, 160000, streams=2)
    assert len(tr.graphs) == 2
    bad = []
    for r in range(12):
        tr.audio.zero_()
        tr.audio.copy_(audio)
        tr.step()
        got = token_lists(*tr.collect())
        bad += [(r, i) for i in range(32) if got[i] != ref[i]]
    assert not bad, f"(replay, clip) with tokens different from the reference: {bad[:12]}"


def _bits(t):
    return t.contiguous().view(torch.int32)


def test_two_one_clip_groups_match_eager(model):
    """Two utterance groups of ONE clip each (the world-1 layout of test_distributed_gpu.py; the
    chunk-parallel scan runs at B = 1) replayed concurrently 40 times: tokens equal eager's."""
    from velocity_asr.pipeline import GraphedTranscriber, audio_to_token_ids, token_lists
    audio = torch.from_numpy(S.make_audio(2, 160000, seed=1234)).to(DEV)
    with torch.no_grad():
        exp = token_lists(*audio_to_token_ids(model, audio))
    tr = GraphedTranscriber(model, 2, 160000, streams=2)
    tr.audio.copy_(audio)
    bad = []
    for r in range(40):
        tr.step()
        got = token_lists(*tr.collect())
        bad += [(r, i) for i in range(2) if got[i] != exp[i]]
    assert not bad, f"(replay, clip) with tokens different from eager: {bad[:12]}"


def test_two_one_clip_groups_stress_800_replays(model):
    """The same two concurrent 1-clip groups, 800 replays, each replay's token block and lengths
    compared with eager's on the device (the race the removed SERIAL_MAX_GROUP fallback covered
    showed in about 1 of 100-200 replays; profiles/r04ah/ ran 800 and 2,000)."""
    from velocity_asr.pipeline import GraphedTranscriber, audio_to_token_ids
    audio = torch.from_numpy(S.make_audio(2, 160000, seed=4321)).to(DEV)
    with torch.no_grad():
        et, el = audio_to_token_ids(model, audio)
    valid = torch.arange(et.shape[1], device=DEV)[None, :] < el[:, None]  # slots past a length are unspecified
    et = et.masked_fill(~valid, 0)
    tr = GraphedTranscriber(model, 2, 160000, streams=2)
    tr.audio.copy_(audio)
    bad = []
    for r in range(800):
        tr.step()
        t, n = tr.collect()
        if not (torch.equal(n, el) and torch.equal(t.masked_fill(~valid, 0), et)):
            bad.append(r)
    assert not bad, f"{len(bad)} of 800 replays differ from eager (first: {bad[:8]})"


def test_scan_beside_coresident_gemms_is_bitwise_alone(model):
    """The local-block scan of 16 clips (the bench's group shape) launched 24 times on one stream
    while a tile-engine GEMM (M = 8016, N = 384) and the 16-row global tail run on another:
    every output bitwise equal to the scan alone."""
    from velocity_asr import audio as A
    from velocity_asr import ops
    audio = torch.from_numpy(S.make_audio(16, 160000, seed=1234)).to(DEV)
    blk, gblk = model.local_ssm.layers[0], model.global_context.global_ssm.layers[0]
    with torch.no_grad():
        mel = A.mel_on_device(audio, frame_pad=1)
        x = model.temporal_binding(mel).contiguous()
        B, L, D = x.shape
        u = ops.ln_dwconv(x, blk.norm1.weight, blk.norm1.bias, blk.conv.weight.view(D, -1), blk.conv.bias,
                          blk.norm1.eps).view(B * L, D)
        xz, xdt = blk.ssm.project(u)
        ref = _bits(blk.ssm.scan(xz, xdt, B, L)).clone()
        g16 = torch.randn(1024, 384, device=DEV)
        x16 = torch.randn(1024, 192, device=DEV)
        sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
        main = torch.cuda.current_stream()
        sa.wait_stream(main)
        sb.wait_stream(main)
        outs = []
        for _ in range(24):
            with torch.cuda.stream(sa):
                ops.gemm(u, model.local_ssm.layers[1].ffn[0].weight, model.local_ssm.layers[1].ffn[0].bias)
                gblk.tail(g16, x16, 16, 64)
            with torch.cuda.stream(sb):
                outs.append(blk.ssm.scan(xz, xdt, B, L))
        main.wait_stream(sa)
        main.wait_stream(sb)
        torch.cuda.synchronize()
    bad = [i for i, o in enumerate(outs) if not torch.equal(_bits(o), ref)]
    assert not bad, f"scan launches {bad} differ from the scan alone"


def test_autotuned_schedule_matches_eager(model):
    """pipeline.autotuned_transcriber builds one graph and two concurrent group graphs for 8 clips,
    keeps the faster: its tokens equal eager's, and the timings it reports cover both."""
    from velocity_asr.pipeline import audio_to_token_ids, autotuned_transcriber, token_lists
    audio = torch.from_numpy(S.make_audio(8, 48000, seed=77)).to(DEV)
    with torch.no_grad():
        exp = token_lists(*audio_to_token_ids(model, audio))
    tr, tried = autotuned_transcriber(model, 8, 48000, reps=2, rounds=1, audio=audio)
    assert sorted(tried) == [1, 2] and len(tr.graphs) in (1, 2)
    assert torch.equal(tr.audio, audio)  # timed on (and holding) the clips it serves
    assert len(tr.autotune_rounds) >= 1 and all(sorted(r) == [1, 2] for r in tr.autotune_rounds)
    assert not getattr(tr, "_candidates", None)  # the losers are freed by default
    tr2, _ = autotuned_transcriber(model, 8, 48000, reps=2, rounds=1, audio=audio, keep_candidates=True)
    assert len(tr2._candidates) == 1  # bench.py's opt-in: kept until release_candidates()
    tr2.release_candidates()
    assert not getattr(tr2, "_candidates", None)
    del tr2
    for _ in range(3):
        tr.step()
        assert token_lists(*tr.collect()) == exp
