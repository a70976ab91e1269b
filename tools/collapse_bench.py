"""Launch-timed vasr_ctc_collapse_keys (argmax keys -> greedy CTC tokens, one launch) on synthetic keys,
library from VASR_LIB; prints a digest of the outputs so builds can be compared.
    python tools/collapse_bench.py [B:L,...]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr import _lib  # noqa: E402


def main():
    shapes = [tuple(int(v) for v in s.split(":")) for s in (sys.argv[1] if len(sys.argv) > 1 else "32:501").split(",")]
    lib = _lib.lib()
    name = os.path.basename(os.environ.get("VASR_LIB", "HEAD"))
    slots = 32
    for B, L in shapes:
        g = torch.Generator(device="cuda").manual_seed(B * 7 + L)
        # keys: (value bits << 32) | (2^32 - 1 - column), 50 / 50 blank (column 0) or a small vocabulary
        val = torch.randint(0, 1 << 30, (B * L, slots), device="cuda", generator=g, dtype=torch.int64)
        col = torch.randint(0, 8, (B * L, slots), device="cuda", generator=g, dtype=torch.int64)
        keys = (val << 32) | (0xFFFFFFFF - col)
        toks = torch.empty(B, L, dtype=torch.int32, device="cuda")
        lens = torch.empty(B, dtype=torch.int32, device="cuda")
        pred = torch.empty(B, L, dtype=torch.int32, device="cuda")

        def run():
            rc = lib.vasr_ctc_collapse_keys(ctypes.c_void_p(keys.data_ptr()), slots, slots, B, L, None, 0, 1,
                                            ctypes.c_void_p(pred.data_ptr()), ctypes.c_void_p(toks.data_ptr()),
                                            ctypes.c_void_p(lens.data_ptr()), None, None, None)
            assert rc == 0, _lib.lib().vasr_last_error()
        run()
        torch.cuda.synchronize()
        valid = torch.arange(L, device="cuda")[None, :] < lens[:, None]
        digest = (int(lens.sum()), int(toks.long().masked_fill(~valid, 0).sum()), int(pred.long().sum()))
        best = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(20):
                run()
            b.record()
            torch.cuda.synchronize()
            best.append(a.elapsed_time(b) * 1e3 / 20)
        print(f"{name:14s} B={B} L={L}: {min(best):.2f} us (median {sorted(best)[2]:.2f})  digest {digest}", flush=True)


if __name__ == "__main__":
    main()
