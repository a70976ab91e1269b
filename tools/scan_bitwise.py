#!/usr/bin/env python3
"""Bitwise A/B of the scan kernels between two builds of the library (VASR_LIB).

    python tools/scan_bitwise.py dump <out.npz>        # with VASR_LIB=<lib>: outputs of every case
    python tools/scan_bitwise.py compare <a.npz> <b.npz>

Cases: streaming scan in modes 0 / 1 / 2 with both lane layouts and both chunk lengths, the
chunk-parallel form (modes 0 / 2), N in {16, 32, 64, 128}, ragged and long L, B in {1, 3, 16}.
A kernel change meant to keep the float operations (instruction selection, data movement)
must leave every output bit unchanged.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "velocity-asr_amd"))


def cases():
    for N, Di in ((16, 64), (32, 384), (64, 384), (128, 256)):
        for B, L in ((1, 1), (1, 17), (3, 501), (1, 1501), (16, 501), (2, 4100)):
            if N == 128 and L > 1501:
                continue
            for mode in (0, 1, 2):
                for npl in ((4,) if N == 128 else (2, 4)):
                    for tc in ((16,) if mode == 1 else (16, 32)):
                        yield ("streaming", N, Di, B, L, mode, npl, tc)
                if mode != 1 and L > 1 and B <= 3:
                    for npl in ((4,) if N == 128 else (2, 4)):
                        yield ("chunked", N, Di, B, L, mode, npl, 16)


def _lib_direct():
    """The library under test (VASR_LIB or the in-tree build) through ctypes alone, so libraries of
    other ABI versions (e.g. the round-start build) dump the same cases: only the scan entry points
    and vasr_set_option, whose signatures every ABI since 12 shares."""
    import ctypes
    path = os.environ.get("VASR_LIB") or os.path.join(REPO, "velocity-asr_amd", "velocity_asr", "lib", "libvasr_hip.so")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    c_p, c_i64, c_i = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.vasr_ssm_scan_f32.argtypes = [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_i64] + [c_i] * 5 + [c_p]
    lib.vasr_ssm_scan_chunked_f32.argtypes = ([c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_i64] + [c_i] * 5
                                              + [c_p, c_i64, c_p])
    lib.vasr_ssm_scan_workspace_floats.argtypes = [c_i] * 4
    lib.vasr_ssm_scan_workspace_floats.restype = c_i64
    lib.vasr_set_option.argtypes = [c_i, c_i]
    lib.vasr_set_option.restype = c_i
    return lib


def dump(path):
    import torch
    lib = _lib_direct()
    OPT_SCAN_LANES, OPT_SCAN_CHUNK = 0, 1  # enum vasr_option (include/vasr.h)
    out = {}
    for form, N, Di, B, L, mode, npl, tc in cases():
        g = torch.Generator(device="cuda").manual_seed(1000 * N + 7 * L + B)
        M = B * L
        xz = torch.randn(M, 2 * Di, device="cuda", generator=g)
        dt = torch.nn.functional.softplus(torch.randn(M, Di, device="cuda", generator=g) - 1)
        bc = torch.randn(M, 2 * N, device="cuda", generator=g)
        A2 = -(torch.arange(1, N + 1, device="cuda", dtype=torch.float32)
               + 0.1 * torch.rand(N, device="cuda", generator=g)) * 1.4426950408889634
        D = 1 + 0.1 * torch.randn(Di, device="cuda", generator=g)
        y = torch.empty(M, Di, device="cuda")
        p0 = lib.vasr_set_option(OPT_SCAN_LANES, npl)
        p1 = lib.vasr_set_option(OPT_SCAN_CHUNK, tc)
        args = (xz.data_ptr(), 2 * Di, dt.data_ptr(), Di, bc.data_ptr(), 2 * N, A2.data_ptr(), D.data_ptr(),
                y.data_ptr(), Di, B, L, Di, N, mode)
        try:
            if form == "chunked":
                nws = lib.vasr_ssm_scan_workspace_floats(B, L, Di, N)
                ws = torch.empty(max(nws, 4), device="cuda")
                rc = lib.vasr_ssm_scan_chunked_f32(*args, ws.data_ptr(), nws, None)
            else:
                rc = lib.vasr_ssm_scan_f32(*args, None)
        finally:
            lib.vasr_set_option(OPT_SCAN_LANES, p0)
            lib.vasr_set_option(OPT_SCAN_CHUNK, p1)
        assert rc == 0, (form, N, Di, B, L, mode, npl, tc, rc)
        torch.cuda.synchronize()
        out["|".join(map(str, (form, N, Di, B, L, mode, npl, tc)))] = y.cpu().numpy()
    np.savez(path, **out)
    print(f"{len(out)} cases -> {path}")


def compare(a, b):
    A, Bz = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        x, y = A[k], Bz[k]
        same = np.array_equal(x.view(np.uint32), y.view(np.uint32))
        if not same:
            bad += 1
            d = np.abs(x - y)
            print(f"DIFF {k}: {int((x.view(np.uint32) != y.view(np.uint32)).sum())} elements, max |d| {d.max():.3e}")
    print(f"{len(A.files) - bad}/{len(A.files)} cases bitwise equal")
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(1 if compare(sys.argv[2], sys.argv[3]) else 0)
