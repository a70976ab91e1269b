"""Graph-timed LayerNorm + adaptive pool: the two launches vs vasr_ln_adaptive_pool_f32 (one), outputs
compared bitwise.  Library from VASR_LIB (velocity_asr._lib), so builds can be A/B'd in turn.
    python tools/lnpool_bench.py [B:L:K,...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr import ops  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from frontend_bench import timed  # noqa: E402


def main():
    shapes = [tuple(int(v) for v in s.split(":")) for s in (sys.argv[1] if len(sys.argv) > 1 else "32:64:16").split(",")]
    lib = os.path.basename(os.environ.get("VASR_LIB", "HEAD"))
    for B, L, K in shapes:
        C = 192
        g = torch.Generator(device="cuda").manual_seed(B + L + K)
        x = torch.randn(B, L, C, device="cuda", generator=g)
        w, b = 1 + 0.1 * torch.randn(C, device="cuda", generator=g), 0.1 * torch.randn(C, device="cuda", generator=g)
        ref = ops.adaptive_pool(ops.layer_norm(x, w, b, 1e-5), K)
        assert torch.equal(ops.ln_adaptive_pool(x, w, b, 1e-5, K), ref), "mismatch"
        t2 = [timed(lambda: ops.adaptive_pool(ops.layer_norm(x, w, b, 1e-5), K)) for _ in range(3)]
        t1 = [timed(lambda: ops.ln_adaptive_pool(x, w, b, 1e-5, K)) for _ in range(3)]
        print(f"{lib:14s} B={B} L={L} K={K}: two launches {min(t2):.2f} us, fused {min(t1):.2f} us", flush=True)


if __name__ == "__main__":
    main()
