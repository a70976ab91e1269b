"""CTC prefix beam search (reference decode.py:128-217; SURVEY §8 f rank 4) against goldens
made by the reference (tests/golden/beam.json, gen_goldens.py::gen_beam).

Bar: token prefixes identical (integer output) and scores within 1e-4 absolute: the scores
are float64 sums of float32 log-softmax values whose last ulps depend on the exp/log
implementation (torch CPU vs numpy vs the device's), over up to 64 frames.
"""

import numpy as np
import pytest
import torch

from conftest import golden_json
from oracle import velocity_ref as R


def _cases():
    g = golden_json("beam.json")
    d = golden_json("decode.json")["cases"]
    for name, c in g["cases"].items():
        lg = np.array(c["logits"] if c["logits"] is not None else d[name]["logits"], np.float32)
        if lg.size == 0:
            lg = lg.reshape(1, 0, 5)
        for w, beams in c["beams"].items():
            yield name, lg, int(w), beams


def _check(got, want):
    assert len(got) == len(want)
    for gb, wb in zip(got, want):
        assert [t for t, _ in gb] == [t for t, _ in wb]
        np.testing.assert_allclose([s for _, s in gb], [s for _, s in wb], atol=1e-4, rtol=0)


@pytest.mark.parametrize("name,lg,w,beams", list(_cases()), ids=lambda v: v if isinstance(v, (str, int)) else "")
def test_oracle_beam_vs_reference(name, lg, w, beams):
    _check(R.ctc_beam_search(lg, w), beams)


@pytest.mark.gpu
@pytest.mark.parametrize("name,lg,w,beams", list(_cases()), ids=lambda v: v if isinstance(v, (str, int)) else "")
def test_device_beam_vs_reference(name, lg, w, beams):
    from velocity_asr import _lib
    from velocity_asr.decode import ctc_beam_search
    _lib.require_device()
    res = ctc_beam_search(torch.from_numpy(lg).cuda(), beam_width=w)
    _check([[(r.tokens, r.score) for r in rb] for rb in res], beams)


@pytest.mark.gpu
def test_device_beam_on_model_logits():
    """Model-sized search (V = 1000, L = 151): device == oracle restatement."""
    from velocity_asr import _lib
    from velocity_asr.decode import ctc_beam_search
    from conftest import golden
    _lib.require_device()
    lg = golden("fwd_b2_3s.npz")["logits"]
    res = ctc_beam_search(torch.from_numpy(lg).cuda(), beam_width=4)
    _check([[(r.tokens, r.score) for r in rb] for rb in res], R.ctc_beam_search(lg, 4))
