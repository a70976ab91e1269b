"""Every BASELINE config's bench workload pinned to the reference.

bench.py rank r transcribes make_audio(32, 160000, seed=1234 + r) (C2 per rank, C3's 256 clips
over 8 ranks); C5 is rank 0's batch through the INT8 fake-quant model.  Goldens:
tests/golden/fwd_fullbatch.npz (rank 0 fp32, and C4's 32 clips at 30 s) and
tests/golden/fwd_benchsets.npz (ranks 1..7 fp32, ranks 0..7 bf16, rank 0 INT8), the reference
CPU path run in chunks of 8 by tests/golden/gen_goldens.py::gen_benchsets.

Bars:
  * fp32: every clip's greedy token list IDENTICAL to the reference (north_star).
  * bf16 model (C3): token edit rate <= 5 % against the fp32 reference (SURVEY §8 d) and against
    the reference's own bf16 run (which drifts 2.2-2.5 % from fp32 on these batches).
  * INT8 (C5): token edit rate <= 5 % against the reference's INT8 run with the same calibration
    (the intended-semantics QAT model; whole-model INT8 is statistical, see test_int8.py).
The measured rates go to $VASR_PARITY_LOG (conftest.record_metric).
"""
import json

import numpy as np
import pytest
import torch

from conftest import golden, record_metric, token_edit_rate
from velocity_asr import synthetic as S

pytestmark = pytest.mark.gpu
DEV = "cuda"
EDIT_BOUND = 0.05


@pytest.fixture(scope="module")
def va():
    import velocity_asr
    from velocity_asr import _lib
    _lib.require_device()
    _lib.load()
    return velocity_asr


@pytest.fixture(scope="module")
def fp32_model(va):
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    return m.to(DEV).eval()


@pytest.fixture(scope="module")
def bf16_model(va):
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    return m.to(DEV).to(torch.bfloat16).eval()


@pytest.fixture(scope="module")
def sets():
    return json.loads(str(golden("fwd_benchsets.npz")["greedy"]))


@pytest.fixture(scope="module")
def full():
    return json.loads(str(golden("fwd_fullbatch.npz")["greedy"]))


def _lists(model, audio):
    from velocity_asr.pipeline import audio_to_token_ids, token_lists
    with torch.no_grad():
        return token_lists(*audio_to_token_ids(model, torch.from_numpy(audio).to(DEV)))


def _fp32_ref(rank, sets, full):
    return full["c2"] if rank == 0 else sets[f"fp32_r{rank}"]


@pytest.mark.parametrize("rank", range(8))
def test_fp32_rank_batches_identical(va, fp32_model, sets, full, rank):
    """C2 at N = 8: each rank's 32 clips, token lists identical to the reference."""
    got = _lists(fp32_model, S.make_audio(32, 160000, seed=1234 + rank))
    ref = _fp32_ref(rank, sets, full)
    bad = [i for i, (a, b) in enumerate(zip(got, ref)) if a != b]
    assert not bad, f"rank {rank}: clips {bad} differ from the reference"


def test_c4_30s_batch_identical(va, fp32_model, full):
    """C4: all 32 x 30 s clips in one B = 32 launch (the reference run in chunks of 4)."""
    got = _lists(fp32_model, S.make_audio(32, 480000, seed=1234))
    bad = [i for i, (a, b) in enumerate(zip(got, full["c4"])) if a != b]
    assert len(full["c4"]) == 32 and not bad, f"C4 clips {bad} differ from the reference"


@pytest.mark.parametrize("rank", range(8))
def test_bf16_rank_batches_edit_rate(va, bf16_model, sets, full, rank):
    """C3 = 256 clips over 8 ranks through the bf16 model (model.to(torch.bfloat16))."""
    got = _lists(bf16_model, S.make_audio(32, 160000, seed=1234 + rank))
    e32 = token_edit_rate(got, _fp32_ref(rank, sets, full))
    eb = token_edit_rate(got, sets[f"bf16_r{rank}"])
    ref_drift = token_edit_rate(sets[f"bf16_r{rank}"], _fp32_ref(rank, sets, full))
    record_metric("bf16_token_edit_rate", rank=rank, vs_fp32_reference=e32, vs_bf16_reference=eb,
                  reference_bf16_vs_fp32=ref_drift)
    print(f"rank {rank}: bf16 edit rate vs fp32 ref {e32:.4f}, vs bf16 ref {eb:.4f} (ref drift {ref_drift:.4f})")
    assert e32 <= EDIT_BOUND and eb <= EDIT_BOUND


def test_int8_bench_batch_edit_rate(va, sets, full):
    """C5: bench.py's INT8 model (prepare_model_for_qat, calibrate_from_activations on
    make_audio(2, 48000, seed=71)) on rank 0's 32 clips."""
    from velocity_asr import compute_mel_spectrogram
    from velocity_asr import quantize as Q
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = Q.prepare_model_for_qat(m.to(DEV).eval()).to(DEV).eval()
    Q.calibrate_from_activations(m, compute_mel_spectrogram(torch.from_numpy(S.make_audio(2, 48000, seed=71)).to(DEV)))
    got = _lists(m, S.make_audio(32, 160000, seed=1234))
    e8 = token_edit_rate(got, sets["int8_r0"])
    e32 = token_edit_rate(got, full["c2"])
    record_metric("int8_token_edit_rate", vs_int8_reference=e8, vs_fp32_reference=e32,
                  reference_int8_vs_fp32=token_edit_rate(sets["int8_r0"], full["c2"]))
    print(f"int8 edit rate vs int8 ref {e8:.4f}, vs fp32 ref {e32:.4f}")
    assert e8 <= EDIT_BOUND
