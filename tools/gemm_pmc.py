"""Launch each projection-GEMM shape of the bench step in isolation, in a fixed order, for
rocprofv3 counter passes (tools/pmc_mfma.sh).  The shapes are the bench's 16-clip launches
(M = 16 x 501 = 8016 token rows) of the split-bf16 engine with the model's epilogues; every
shape runs REPS launches after a warm-up, separated by synchronize, so dispatch k of the
gemm kernels belongs to shape k // REPS.  Writes the order to gpurun_out/gemm_pmc_order.json.
Usage (GPU box): python tools/gemm_pmc.py [M]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr import _lib, ops  # noqa: E402

REPS = 6
# (name, N, K, epilogue, lda): the SSM block (ssm.py), the CTC head with the fused argmax
SHAPES = [("in_proj", 768, 192, "none", None), ("x_dt", 512, 384, "softplus", 768),
          ("out_proj", 192, 384, "residual", None), ("ffn1", 384, 192, "gelu", None),
          ("ffn2", 192, 384, "residual", None), ("head_argmax", 1000, 192, "argmax", None)]


def main():
    _lib.require_device()
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 8016
    E = {"none": _lib.EPI_NONE, "softplus": _lib.EPI_SOFTPLUS_FROM, "residual": _lib.EPI_RESIDUAL,
         "gelu": _lib.EPI_GELU}
    g = torch.Generator(device="cuda").manual_seed(0)
    order = []
    for name, N, K, epi, lda in SHAPES:
        a = torch.randn(M, lda or K, device="cuda", generator=g)[:, :K]
        w = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
        b = torch.randn(N, device="cuda", generator=g)
        kw = {}
        if epi == "softplus":
            kw["n_out"] = 128
        if epi == "residual":
            kw["aux"] = torch.randn(M, N, device="cuda", generator=g)
        if epi == "argmax":
            def fn():
                return ops.gemm_argmax(a, w, b)
        else:
            def fn():
                return ops.gemm(a, w, b, epilogue=E[epi], **kw)
        fn()  # builds the split weights outside the counted launches
        torch.cuda.synchronize()
        for _ in range(REPS):
            fn()
            torch.cuda.synchronize()
        order.append(dict(name=name, M=M, N=N, K=K, epilogue=epi, reps=REPS,
                          flops=2.0 * M * N * K, bf16_products=6))
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/gemm_pmc_order_{M}.json", "w") as f:
        json.dump(order, f, indent=1)
    print(json.dumps(order))


if __name__ == "__main__":
    main()
