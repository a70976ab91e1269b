"""scripts/transcribe.py and scripts/evaluate.py: host logic on CPU, end to end on the GPU.

The end-to-end cases write the golden clips as float32 WAV files (lossless), save the
seeded model as a reference-format checkpoint, run the scripts' main() and compare the
transcripts with the reference's own greedy decode of the same clips (tests/golden).
"""

import importlib.util
import json
import os

import numpy as np
import pytest
import torch

from conftest import PKG_ROOT, golden, golden_json
from velocity_asr import synthetic as S


def _script(name):
    spec = importlib.util.spec_from_file_location(f"vasr_script_{name}", os.path.join(PKG_ROOT, "scripts", f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_float_wav_roundtrip_exact(tmp_path):
    import velocity_asr as v
    from velocity_asr.audio import write_wav
    x = S.make_audio(2, 3001, seed=3)
    write_wav(str(tmp_path / "a.wav"), x)
    np.testing.assert_array_equal(v.load_audio(str(tmp_path / "a.wav"), mono=False).numpy(), x)
    write_wav(str(tmp_path / "m.wav"), x[0])
    np.testing.assert_array_equal(v.load_audio(str(tmp_path / "m.wav")).numpy(), x[0])
    (tmp_path / "bad.wav").write_bytes(b"RIFF\0\0\0\0WAVX")
    with pytest.raises(ValueError):
        v.load_audio(str(tmp_path / "bad.wav"))


def test_group_words_follows_reference_convention():
    from velocity_asr import create_default_vocabulary
    from velocity_asr.transcription import frames_to_seconds, group_words
    voc = create_default_vocabulary(100)
    a, b, sp = voc.index("a"), voc.index("b"), voc.index(" ")
    toks = [a, b, sp, sp, b, 999]
    spans = [(0, 1), (2, 2), (3, 5), (6, 6), (7, 8), (9, 12)]
    words = group_words(toks, spans, voc)
    # a word ends at its closing separator's end frame; the last at the final token's end
    assert words == [{"word": "ab", "start": 0.0, "end": frames_to_seconds(5)},
                     {"word": "b<unk>", "start": frames_to_seconds(7), "end": frames_to_seconds(12)}]
    assert frames_to_seconds(50) == 1.0
    assert group_words([], [], voc) == [] and group_words([sp], [(0, 0)], voc) == []


def test_manifest_and_listing(tmp_path):
    from velocity_asr.transcription import find_audio_files, load_manifest
    (tmp_path / "d").mkdir()
    for n in ("x.wav", "d/y.FLAC", "z.txt"):
        (tmp_path / n).write_bytes(b"")
    assert sorted(p.name for p in find_audio_files(str(tmp_path))) == ["x.wav", "y.FLAC"]
    m = tmp_path / "m.tsv"
    m.write_text("x.wav\thello world\n\n/abs/y.wav\tb\n", encoding="utf-8")
    assert load_manifest(str(m)) == [(str(tmp_path / "x.wav"), "hello world"), ("/abs/y.wav", "b")]
    assert load_manifest(str(tmp_path / "missing.tsv")) == []


def test_script_arguments():
    tr, ev = _script("transcribe"), _script("evaluate")
    a = tr.parse_args(["f.wav", "--checkpoint", "c.pt", "--timestamps", "--format", "json", "-q"])
    assert (a.audio, a.timestamps, a.format, a.quiet, a.device) == ("f.wav", True, "json", True, "cuda")
    with pytest.raises(SystemExit):
        tr.parse_args(["--checkpoint", "c.pt"])
    with pytest.raises(SystemExit):
        ev.parse_args(["--checkpoint", "c.pt"])
    assert ev.parse_args(["--checkpoint", "c.pt", "--audio-dir", "d", "--beam-width", "4"]).beam_width == 4


# --------------------------------------------------------------------------- on the GPU
@pytest.fixture(scope="module")
def ckpt_and_clips(tmp_path_factory):
    import velocity_asr as v
    from velocity_asr.audio import write_wav
    root = tmp_path_factory.mktemp("scripts")
    m = v.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(x) for k, x in S.make_weights(None, seed=0).items()})
    m.save_pretrained(str(root / "model.pt"))
    clips = root / "clips"
    clips.mkdir()
    a = S.make_audio(2, 48000, seed=21)          # fwd_b2_3s golden clips (equal length: one batch)
    write_wav(str(clips / "c0.wav"), a[0])
    write_wav(str(clips / "c1.wav"), a[1])
    write_wav(str(clips / "e.wav"), S.make_audio(1, 16333, seed=35)[0])  # fwd_edge golden clip
    return root, clips


def _expected_texts():
    import velocity_asr as v
    from oracle import velocity_ref as R
    dec = v.CTCDecoder(v.create_default_vocabulary(1000))
    b2 = golden_json("decode_fwd.json")["results"]["b2_3s"]
    edge = R.ctc_greedy_decode(golden("fwd_edge.npz")["S16333__logits"])[0]
    return {"c0.wav": dec._tokens_to_text(b2[0]), "c1.wav": dec._tokens_to_text(b2[1]),
            "e.wav": dec._tokens_to_text(edge)}


@pytest.mark.gpu
def test_transcribe_script_dir_json(ckpt_and_clips, tmp_path):
    root, clips = ckpt_and_clips
    tr = _script("transcribe")
    out = tmp_path / "all.json"
    assert tr.main([ "--checkpoint", str(root / "model.pt"), "--input-dir", str(clips), "--output-dir",
                    str(tmp_path / "per"), "--format", "json", "--output", str(out), "-q"]) == 0
    res = {os.path.basename(r["file"]): r for r in json.loads(out.read_text())}
    exp = _expected_texts()
    assert {k: r["transcription"] for k, r in res.items()} == exp
    assert res["c0.wav"]["duration"] == 3.0
    per = json.loads((tmp_path / "per" / "e.json").read_text())
    assert per["transcription"] == exp["e.wav"]


@pytest.mark.gpu
def test_transcribe_script_single_file_timestamps(ckpt_and_clips, tmp_path, capsys):
    from velocity_asr import create_default_vocabulary
    from velocity_asr.transcription import group_words
    root, clips = ckpt_and_clips
    tr = _script("transcribe")
    assert tr.main([str(clips / "c1.wav"), "--checkpoint", str(root / "model.pt"), "--timestamps",
                    "--format", "json", "-q"]) == 0
    r = json.loads(capsys.readouterr().out)
    toks, spans = golden_json("decode_fwd.json")["results"]["b2_3s_ts"][1]
    words = group_words(toks, [tuple(s) for s in spans], create_default_vocabulary(1000))
    assert r["words"] == words
    assert r["transcription"] == " ".join(w["word"] for w in words)


@pytest.mark.gpu
def test_evaluate_script_manifest_and_dir(ckpt_and_clips, tmp_path, capsys):
    root, clips = ckpt_and_clips
    ev = _script("evaluate")
    exp = _expected_texts()
    man = tmp_path / "m.tsv"
    man.write_text("".join(f"{clips / k}\t{t}\n" for k, t in exp.items()), encoding="utf-8")
    out = tmp_path / "report.txt"
    assert ev.main(["--checkpoint", str(root / "model.pt"), "--test-set", str(man), "--output", str(out)]) == 0
    assert "WER: 0.00%" in out.read_text() and "Samples: 3" in out.read_text()
    out2 = tmp_path / "dir.tsv"
    assert ev.main(["--checkpoint", str(root / "model.pt"), "--audio-dir", str(clips), "--output", str(out2)]) == 0
    rows = dict(line.split("\t", 1) for line in out2.read_text().splitlines())
    assert rows == exp


@pytest.mark.gpu
@pytest.mark.parametrize("clip", ["clip_2s.wav", "chirp_3s.wav", "clip_10s.wav"])
def test_transcribe_script_matches_reference_cli_output(ckpt_and_clips, tmp_path, capsys, clip):
    """scripts/transcribe.py --format json [--timestamps] vs the reference's own
    transcribe_file output for the same clip and weights (tests/golden/cli_transcribe.json,
    captured from /root/reference/scripts/transcribe.py in the build container)."""
    from velocity_asr.audio import write_wav
    root, _ = ckpt_and_clips
    g = golden_json("cli_transcribe.json")["clips"][clip]
    recipe = g["recipe"]
    make = {"make_audio(1, 32000, seed=91)[0]": lambda: S.make_audio(1, 32000, seed=91)[0],
            "make_chirp(48000)": lambda: S.make_chirp(48000),
            "make_audio(2, 160000, seed=1234)[1]": lambda: S.make_audio(2, 160000, seed=1234)[1]}[recipe]
    path = tmp_path / clip
    write_wav(str(path), make())
    tr = _script("transcribe")
    for key, extra in (("text", []), ("timestamps", ["--timestamps"])):
        assert tr.main([str(path), "--checkpoint", str(root / "model.pt"), "--format", "json", "-q"] + extra) == 0
        got = json.loads(capsys.readouterr().out)
        exp = dict(g[key], file=str(path))
        assert got == exp, key


def test_batches_group_equal_lengths_without_ragged_front_end():
    """without per-length kernels (VASR_STFT=gemm, n_mels > 85) a batch holds clips of
    one sample count; with them, up to batch_size clips of any length."""
    from velocity_asr.transcription import _batches
    items = [(i, torch.zeros(n)) for i, n in enumerate([500, 500, 500, 800, 900, 900, 900, 900, 1200])]
    lens = lambda bs: [[it[1].numel() for it in b] for b in bs]  # noqa: E731
    assert lens(_batches(items, 3, True)) == [[500, 500, 500], [800, 900, 900], [900, 900, 1200]]
    assert lens(_batches(items, 3, False)) == [[500, 500, 500], [800], [900, 900, 900], [900], [1200]]
    assert lens(_batches(items, 16, False)) == [[500, 500, 500], [800], [900, 900, 900, 900], [1200]]
    assert list(_batches([], 4, False)) == []


@pytest.mark.gpu
def test_transcribe_files_mixed_lengths_128_mels(tmp_path):
    """a model with mel_bins = 128 (no per-length front end) over files of different
    lengths: no file errors, and every file's text equals its transcription alone."""
    import velocity_asr as v
    from velocity_asr.audio import write_wav
    from velocity_asr.transcription import transcribe_files
    cfg = dict(mel_bins=128, d_model=96, ssm_layers=2, ssm_state_dim=32, global_ssm_state_dim=16,
               attention_heads=2, attention_dim=24, vocab_size=50)
    W = S.make_weights(cfg, seed=5)
    m = v.VELOCITYASR(v.VelocityASRConfig(**cfg))
    m.load_state_dict({k: torch.from_numpy(w) for k, w in W.items()}, strict=True)
    m = m.to("cuda").eval()
    dec = v.CTCDecoder(v.create_default_vocabulary(50))
    paths = []
    for i, n in enumerate([16000, 24000, 16000, 9000, 24000]):
        p = tmp_path / f"c{i}.wav"
        write_wav(str(p), torch.from_numpy(S.make_audio(1, n, seed=40 + i)[0]), 16000)
        paths.append(p)
    got = transcribe_files(m, paths, dec, "cuda", batch_size=4)
    assert all("error" not in r for r in got), got
    for p, r in zip(paths, got):
        alone = transcribe_files(m, [p], dec, "cuda", batch_size=1)[0]
        assert r == alone
