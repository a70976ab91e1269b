import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "velocity-asr_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: longer CPU oracle runs")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def golden_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def default_weights():
    from velocity_asr import synthetic
    return synthetic.make_weights(None, seed=0)


def record_error(got, want, tol):
    """Append {test, max_abs, worst |diff| / (atol + rtol |want|)} to $VASR_PARITY_LOG (JSON lines)
    when it is set: the measured margin of a float comparison, reported in DESIGN.md §4."""
    path = os.environ.get("VASR_PARITY_LOG")
    if not path:
        return
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    d = np.abs(got - want)
    rec = dict(test=os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0],
               max_abs=float(d.max()) if d.size else 0.0,
               max_rel=float((d / np.maximum(np.abs(want), 1e-30)).max()) if d.size else 0.0,
               tol_use=float((d / (tol["atol"] + tol["rtol"] * np.abs(want))).max()) if d.size else 0.0)
    with open(path, "a") as f:
        f.write(json.dumps(rec) + "\n")


def edit_distance(a, b):
    """Levenshtein distance between two token lists (row DP, each row vectorised)."""
    a, b = np.asarray(a, np.int64), np.asarray(b, np.int64)
    if len(b) == 0:
        return len(a)
    ar = np.arange(len(b) + 1)
    prev = ar.copy()
    for i, x in enumerate(a, 1):
        base = np.empty_like(prev)
        base[0] = i
        base[1:] = np.minimum(prev[1:] + 1, prev[:-1] + (b != x))
        prev = np.minimum.accumulate(base - ar) + ar
    return int(prev[-1])


def token_edit_rate(got, ref):
    """Summed edit distance of token lists over the summed reference length (a token-level WER)."""
    return sum(edit_distance(a, b) for a, b in zip(got, ref)) / max(1, sum(len(b) for b in ref))


def record_metric(name, **values):
    """Append {test, name, values} to $VASR_PARITY_LOG when set (measured rates for DESIGN.md)."""
    path = os.environ.get("VASR_PARITY_LOG")
    if not path:
        return
    rec = dict(test=os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0], name=name, **values)
    with open(path, "a") as f:
        f.write(json.dumps(rec) + "\n")
