"""Composed projection GEMM (u @ [W_in; W_xdt W_in_x]^T, softplus on the dt columns) alone, at the
bench's launch shapes: rows engine time per launch (HIP events over back-to-back launches) and
bitwise equality with the tile engine.  Usage (GPU box): python tools/rows_bench.py [M ...]
(VASR_LIB=<variant .so> selects a diagnostic build)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr import _lib, ops  # noqa: E402


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    _lib.require_device()
    Ms = [int(v) for v in sys.argv[1:]] or [8016, 16032]
    g0 = torch.Generator(device="cuda").manual_seed(0)
    w = torch.randn(1280, 192, device="cuda", generator=g0) * 0.07
    b = torch.cat([torch.zeros(896, device="cuda"), torch.randn(384, device="cuda", generator=g0) * 0.1])
    lib = os.environ.get("VASR_LIB", "default")
    for M in Ms:
        u = torch.randn(M, 192, device="cuda", generator=g0)
        out = torch.empty(M, 1280, device="cuda")

        def run():
            return ops.gemm(u, w, b, epilogue=_lib.EPI_SOFTPLUS_FROM, n_out=896, out=out)
        t_rows = timed(run)
        rows = run().clone()
        with ops.option(_lib.OPT_GEMM_ENGINE, 1):
            t_tiles = timed(run)
            tiles = run().clone()
        same = torch.equal(rows.view(torch.int32), tiles.view(torch.int32))
        flops = 6 * 2.0 * M * 1280 * 192
        print(f"lib={os.path.basename(lib)} M={M}: rows {t_rows:.2f} us ({flops / t_rows / 1e6:.0f} bf16-TF/s), "
              f"tiles {t_tiles:.2f} us, bitwise equal {same}", flush=True)
        # the same projection without the 384 z columns (z formed elsewhere):
        # [x | B | C | dt], softplus from column 512
        w_noz = torch.cat([w[:384], w[768:]]).contiguous()
        b_noz = torch.cat([b[:384], b[768:]]).contiguous()
        out_noz = torch.empty(M, 896, device="cuda")

        def run_noz():
            return ops.gemm(u, w_noz, b_noz, epilogue=_lib.EPI_SOFTPLUS_FROM, n_out=512, out=out_noz)
        t_noz = timed(run_noz)
        noz = run_noz()
        same_noz = torch.equal(noz.view(torch.int32), torch.cat([rows[:, :384], rows[:, 768:]], 1).view(torch.int32))
        print(f"lib={os.path.basename(lib)} M={M}: without z (N = 896) rows {t_noz:.2f} us, "
              f"columns bitwise equal to the 1280-column launch's {same_noz}", flush=True)


if __name__ == "__main__":
    main()
