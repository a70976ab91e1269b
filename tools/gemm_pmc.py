"""Launch each projection-GEMM shape of the bench step in isolation, in a fixed order, for
rocprofv3 counter passes (tools/pmc_mfma.sh).  The shapes are the bench's 16-clip launches
(M = 16 x 501 = 8016 token rows) with the model's epilogues; every shape runs REPS launches
after a warm-up, separated by synchronize, so dispatch k of a kernel family belongs to
shape k // (REPS + 1).  Writes the order to gpurun_out/gemm_pmc_order_<M>.json.

Shape sets:
  head (default)  the kernels the HEAD step runs: the composed
                  [in_proj; x_proj.dt_proj] GEMM (N 1280, K 192, softplus from column 768),
                  the CTC head with the fused argmax (N 1000), and the fused SSMBlock tail
                  (ssm_tail_kernel: 32 rows x 12 waves at M = 8016, 16 rows x 4 waves at the
                  global blocks' M = 16 x 64 = 1024)
  split           the pre-composition projection GEMMs (round-2 table)
Usage (GPU box): python tools/gemm_pmc.py [M] [head|split]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr import _lib, ops  # noqa: E402

REPS = 6
# (name, N, K, epilogue, lda): the SSM block (ssm.py), the CTC head with the fused argmax
SPLIT = [("in_proj", 768, 192, "none", None), ("x_dt", 512, 384, "softplus", 768),
         ("out_proj", 192, 384, "residual", None), ("ffn1", 384, 192, "gelu", None),
         ("ffn2", 192, 384, "residual", None), ("head_argmax", 1000, 192, "argmax", None)]
HEAD = [("head_comp", 1280, 192, "softplus", None), ("ctc_argmax", 1000, 192, "argmax", None),
        ("tail", 192, 384, "tail", None), ("tail_global", 192, 384, "tail1024", None),
        # the z-in-tail block (round 6): the projection without z (softplus from column 512) and the
        # tail that forms z itself (ssm_tail_gated_kernel: z product + the three tail products)
        ("head_noz", 896, 192, "softplus", None), ("tail_gated", 192, 384, "tailg", None)]


def main():
    _lib.require_device()
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 8016
    which = sys.argv[2] if len(sys.argv) > 2 else "head"
    E = {"none": _lib.EPI_NONE, "softplus": _lib.EPI_SOFTPLUS_FROM, "residual": _lib.EPI_RESIDUAL,
         "gelu": _lib.EPI_GELU}
    g = torch.Generator(device="cuda").manual_seed(0)
    order = []
    for name, N, K, epi, lda in (HEAD if which == "head" else SPLIT):
        m = 1024 if epi == "tail1024" else M
        # the engine the launcher picks (gemm_rows.hip try_rows_x3: K = 192, N >= 512, M >= 4096,
        # unpaired non-argmax epilogues -> A-rows-stationary; else the LDS-ring tiles)
        rows = K == 192 and N >= 512 and m >= 4096 and epi in ("none", "gelu", "softplus")
        kernel = "gemm_rows_kernel" if rows else "gemm_x3_kernel"
        flops = 2.0 * m * N * K
        if epi == "tailg":
            D, Ei = 192, 384
            yd = torch.randn(m, Ei, device="cuda", generator=g)
            u = torch.randn(m, D, device="cuda", generator=g)
            wz = torch.randn(Ei, D, device="cuda", generator=g) / D ** 0.5
            x = torch.randn(m, D, device="cuda", generator=g)
            wo = torch.randn(D, Ei, device="cuda", generator=g) / Ei ** 0.5
            w1 = torch.randn(Ei, D, device="cuda", generator=g) / D ** 0.5
            w2 = torch.randn(D, Ei, device="cuda", generator=g) / Ei ** 0.5
            lw, lb = torch.ones(D, device="cuda"), torch.zeros(D, device="cuda")
            b1, b2 = torch.randn(Ei, device="cuda", generator=g), torch.randn(D, device="cuda", generator=g)

            def fn():
                return ops.ssm_block_tail_gated(yd, u, wz, 2, x, wo, lw, lb, 1e-5, w1, b1, w2, b2)
            kernel = "ssm_tail_gated_kernel"
            flops = 4 * 2.0 * m * D * Ei  # z, out_proj, ffn1, ffn2
        elif epi.startswith("tail"):
            D, Ei = 192, 384
            gin = torch.randn(m, Ei, device="cuda", generator=g)
            x = torch.randn(m, D, device="cuda", generator=g)
            wo = torch.randn(D, Ei, device="cuda", generator=g) / Ei ** 0.5
            w1 = torch.randn(Ei, D, device="cuda", generator=g) / D ** 0.5
            w2 = torch.randn(D, Ei, device="cuda", generator=g) / Ei ** 0.5
            lw, lb = torch.ones(D, device="cuda"), torch.zeros(D, device="cuda")
            b1, b2 = torch.randn(Ei, device="cuda", generator=g), torch.randn(D, device="cuda", generator=g)

            def fn():
                return ops.ssm_block_tail(gin, x, wo, lw, lb, 1e-5, w1, b1, w2, b2)
            kernel = "ssm_tail_kernel"
            flops = 3 * 2.0 * m * D * Ei  # out_proj, ffn1, ffn2
        else:
            a = torch.randn(m, lda or K, device="cuda", generator=g)[:, :K]
            w = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
            b = torch.randn(N, device="cuda", generator=g)
            kw = {}
            if epi == "softplus":
                kw["n_out"] = {"head_comp": 896, "head_noz": 512}.get(name, 128)
            if epi == "residual":
                kw["aux"] = torch.randn(m, N, device="cuda", generator=g)
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
        order.append(dict(name=name, M=m, N=N, K=K, epilogue=epi, reps=REPS, kernel=kernel,
                          flops=flops, bf16_products=6))
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/gemm_pmc_order_{M}.json", "w") as f:
        json.dump(order, f, indent=1)
    print(json.dumps(order))


if __name__ == "__main__":
    main()
