"""bench.py's validity checks on the host (no GPU): the reference-token check of the timed graphs
(golden_check / golden_summary) and the exit path (run_verdict) on a forced mismatch, and the
schedule description.  VERDICT r04 weak 8: a failed reference check must fail the run."""

import argparse
import json
import os

import numpy as np
import torch

import bench

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _args(**kw):
    a = argparse.Namespace(bf16=False, int8=False, seconds=10.0, batch=32)
    a.__dict__.update(kw)
    return a


def _c2_reference():
    full = json.loads(str(np.load(os.path.join(GOLD, "fwd_fullbatch.npz"), allow_pickle=False)["greedy"]))
    return full["c2"]


def _as_tensors(lists):
    L = max(1, max(len(x) for x in lists))
    toks = torch.zeros((len(lists), L), dtype=torch.int32)
    for b, x in enumerate(lists):
        toks[b, :len(x)] = torch.tensor(x, dtype=torch.int32)
    lens = torch.tensor([len(x) for x in lists], dtype=torch.int32)
    return toks, lens


def test_golden_check_passes_reference_tokens():
    ref = _c2_reference()
    toks, lens = _as_tensors(ref)
    c = bench.golden_check(toks, lens, _args(), rank=0)
    g = bench.golden_summary(c, _args())
    assert g["clips"] == 32 and g["clips_identical"] == 32 and g["all_ranks_pass"]
    assert bench.run_verdict(True, g, g, g) == (0, [])


def test_forced_mismatch_fails_the_run():
    ref = [list(x) for x in _c2_reference()]
    ref[5] = ref[5][:-1] + [ref[5][-1] % 999 + 1]  # one token of one clip changed
    toks, lens = _as_tensors(ref)
    g = bench.golden_summary(bench.golden_check(toks, lens, _args(), rank=0), _args())
    assert g["clips_identical"] == 31 and not g["all_ranks_pass"]
    ok = bench.golden_summary(bench.golden_check(*_as_tensors(_c2_reference()), _args(), rank=0), _args())
    # any one failing check fails the run: timed, warm-up, or eager
    for combo in ((g, ok, ok), (ok, g, ok), (ok, ok, g)):
        rc, why = bench.run_verdict(True, *combo)
        assert rc == 1 and len(why) == 1 and "all_ranks_pass is false" in why[0]
    rc, why = bench.run_verdict(False, ok, ok, ok)
    assert rc == 1 and "graph_tokens_match_eager" in why[0]
    # no golden for this workload (None) is not a failure
    assert bench.run_verdict(True, None, None, None) == (0, [])


def test_schedule_how_reflects_candidates():
    assert "single candidate" in bench.schedule_how({}, 1)
    h = bench.schedule_how({1: 2.1, 2: 2.2}, 1)
    assert "2 schedules" in h and "own audio" in h
    assert "max over ranks" in bench.schedule_how({1: 2.1, 2: 2.2}, 8)
