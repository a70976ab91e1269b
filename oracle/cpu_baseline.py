"""CPU baseline of bench.py (test infrastructure, like the rest of oracle/: only bench.py's
cpu_baseline leg runs it, and never on the timed path).

The reference path restated in numpy (oracle/velocity_ref.py, with the reference's materialised
tree scan, SCAN_FORM = "tree", ssm.py:216-295) on the bench's own clips, one clip per call as the
reference's scripts run it (scripts/transcribe.py:69-78), data-parallel over `workers` spawned
processes of one BLAS thread each -- the host cores granted to the GPU job (OMP_NUM_THREADS: 16
per GPU on the box).  The spawned workers re-import the parent's main module (bench.py imports
torch and numpy) before `_init` runs, so the one-thread BLAS environment is set in the parent
before the pool starts (children inherit it before any import) and `_init` also caps every
loaded BLAS / OpenMP pool with threadpoolctl; each worker reports its BLAS thread count.
Timing: one warm-up clip per worker, then `repeats` passes over the same `clips` clips; the
median pass is reported.
"""
from __future__ import annotations

import importlib.util
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SYN_PATH = os.path.join(REPO, "velocity-asr_amd", "velocity_asr", "synthetic.py")

_state = {}
_THREAD_VARS = ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")


def _blas_threads() -> int:
    """Largest thread count over the BLAS / OpenMP pools loaded in this process."""
    try:
        from threadpoolctl import threadpool_info
        return max([int(p.get("num_threads", 1)) for p in threadpool_info()] or [1])
    except Exception:
        return -1


def _init(seconds: float, seed: int, n: int):
    for v in _THREAD_VARS:
        os.environ[v] = "1"
    try:
        from threadpoolctl import threadpool_limits
        _state["limits"] = threadpool_limits(1)  # pools created before _init (re-imported __main__)
    except Exception:
        pass
    if HERE not in sys.path:
        sys.path.insert(0, REPO)
    spec = importlib.util.spec_from_file_location("vasr_synthetic", SYN_PATH)
    syn = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(syn)
    from oracle import velocity_ref as R
    R.SCAN_FORM = "tree"
    _state.update(R=R, W=syn.make_weights(None, seed=0), cfg=dict(syn.DEFAULT_CONFIG),
                  audio=syn.make_audio(n, int(seconds * 16000), seed=seed))


def _threads(_i: int) -> int:
    return _blas_threads()


def _clip(i: int) -> int:
    R, W, cfg, audio = _state["R"], _state["W"], _state["cfg"], _state["audio"]
    toks = R.ctc_greedy_decode(R.forward(W, R.compute_mel_spectrogram(audio[i:i + 1]), cfg))
    return len(toks[0])


def measure(workers: int = 16, clips: int = 32, seconds: float = 10.0, seed: int = 1234, repeats: int = 3) -> dict:
    """RTFx of the oracle over `clips` clips of make_audio(clips, seconds * 16 kHz, seed)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")  # fresh interpreters: nothing of the parent's HIP state
    workers = max(1, min(workers, clips))
    saved = {v: os.environ.get(v) for v in _THREAD_VARS}
    os.environ.update({v: "1" for v in _THREAD_VARS})  # inherited by the spawned children
    try:
        pool = ctx.Pool(workers, initializer=_init, initargs=(seconds, seed, clips))
    finally:
        for v, old in saved.items():
            if old is None:
                os.environ.pop(v, None)
            else:
                os.environ[v] = old
    with pool:
        blas = max(pool.map(_threads, range(workers), chunksize=1))
        pool.map(_clip, range(workers), chunksize=1)  # warm-up: one clip per worker
        passes = []
        for _ in range(repeats):
            t0 = time.perf_counter()
            pool.map(_clip, range(clips), chunksize=1)
            passes.append(time.perf_counter() - t0)
    med = statistics.median(passes)
    return dict(rtfx=clips * seconds / med, passes_s=[round(p, 2) for p in passes], workers=workers, clips=clips,
                blas_threads_per_worker=blas)
