"""Isolated timings of the front-end launches (no concurrent streams): |STFT|^2 by the real-FFT
kernel vs reflect pad + windowed-DFT GEMM, and the chunked log-mel normalisation (the fused
STFT + log-mel kernel this once timed was removed in round 3).
Usage (GPU box): python tools/frontend_bench.py [B] [S]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr import _lib, audio as A, ops  # noqa: E402


def timed(fn, iters=20, reps=5):
    """Per-call device time from a HIP graph of `iters` calls (no host launch overhead)."""
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (iters * reps)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 160000
    _lib.require_device()
    dev = torch.device("cuda")
    x = torch.randn(B, S, device=dev) * 0.1
    tb = A._tables(dev, 400, 80, 16000)
    F = S // 160 + 1
    ld = (S + 400 + 3) // 4 * 4
    power = torch.empty((B, F, 201), device=dev)

    def fft():
        ops.stft_power_400(x, tb.window)

    def gemm():
        xp = ops.reflect_pad(x, 200, ld)
        ops.gemm_batched(xp, 160, ld, F, B, 400, tb.dft, None, power, 201, F * 201,
                         epilogue=_lib.EPI_PAIR_POWER, n_out=201)

    p = ops.stft_power_400(x, tb.window)

    def mel():
        ops.mel_log_norm(p, 201, F * 201, tb.fb_csr, B, F, 80, True)

    t_fft, t_gemm, t_mel = timed(fft), timed(gemm), timed(mel)
    byt = B * S * 4 + B * F * 201 * 4
    print(f"B={B} S={S} F={F}: stft fft {t_fft:.2f} us ({byt / t_fft / 1e3:.0f} GB/s algorithmic), "
          f"pad+dft gemm {t_gemm:.2f} us, log-mel+norm {t_mel:.2f} us", flush=True)


if __name__ == "__main__":
    main()
