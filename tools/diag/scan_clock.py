#!/usr/bin/env python3
"""The shader clock the streaming scan runs at, from inside the kernel (the 32-clip
scan launch took 96 us in some processes and 108 us in others).

Needs a library built with -DVASR_SCAN_STAMPS (tools/build_variant_lib.sh scan_stamps -DVASR_SCAN_STAMPS),
passed as VASR_LIB: every workgroup of the N = 64 streaming kernel records s_memtime / s_memrealtime at
entry and exit.  Rounds of: `load` bench steps (the C2 graph, one stream), then `reps` back-to-back
scan launches at the C2 shape (as bench.py's isolated_times) timed by HIP events, the last launch's
stamps read back.  Per round: us per launch, the median workgroup's clock (cycles / real time) and
cycles, the launch's first-entry-to-last-exit span.  If a slow round shows the same cycles at a lower
clock, the launch time follows the clock the chip holds (DVFS); if the cycles rise, the kernel's own
execution changed.

    VASR_LIB=tools/_variants/scan_stamps.so python tools/diag/scan_clock.py [rounds] [load] [reps]
"""
import collections
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "velocity-asr_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    load = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    from velocity_asr import _lib, ops
    from velocity_asr import synthetic as S
    from velocity_asr.pipeline import GraphedTranscriber
    import bench
    lib = _lib.lib()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, L, Di, N = 32, 501, 384, 64
    model = bench.build_model(dev)
    tr = GraphedTranscriber(model, B, 160000, dev, streams=1)
    tr.audio.copy_(torch.from_numpy(S.make_audio(B, 160000, seed=1234)).to(dev))
    g = torch.Generator(device="cuda").manual_seed(0)
    M = B * L
    xz = torch.randn(M, 2 * Di, device="cuda", generator=g)
    dt = torch.nn.functional.softplus(torch.randn(M, Di, device="cuda", generator=g) - 1)
    bc = torch.randn(M, 2 * N, device="cuda", generator=g)
    A2 = -torch.arange(1, N + 1, device="cuda", dtype=torch.float32) * 1.4426950408889634
    D = torch.ones(Di, device="cuda")
    out = torch.empty(M, Di, device="cuda")
    nblk = B * (Di // 16)
    stamps = torch.zeros(5 * nblk, device="cuda", dtype=torch.int64)
    f = lib.vasr_diag_scan_stamps
    f.argtypes = [ctypes.c_void_p]
    assert f(ctypes.c_void_p(stamps.data_ptr())) == 0
    t_start = time.time()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    print("round   t_s  load_ms/step  scan_us/launch  clock_GHz(median wg)  cycles_k(median wg)  span_us  xccs")
    for r in range(rounds):
        s.record()
        for _ in range(load):
            tr.step()
        e.record()
        torch.cuda.synchronize()
        step_ms = s.elapsed_time(e) / load
        for _ in range(3):
            ops.ssm_scan(xz, dt, bc, A2, D, B, L, 2, out=out)
        s.record()
        for _ in range(reps):
            ops.ssm_scan(xz, dt, bc, A2, D, B, L, 2, out=out)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / reps * 1e3
        st = stamps.view(nblk, 5).cpu().double()
        cyc = st[:, 3] - st[:, 1]
        real = st[:, 4] - st[:, 2]
        ghz = (cyc / real.clamp(min=1) * 0.1).median().item()
        span = (st[:, 4].max() - st[:, 2].min()).item() / 100.0
        xcc = st[:, 0].long() & 0xF
        print(f"{r:5d} {time.time() - t_start:6.1f} {step_ms:12.3f} {us:15.2f} {ghz:21.3f} {cyc.median().item() / 1e3:20.1f} "
              f"{span:8.1f}  {int(xcc.unique().numel())}", flush=True)
    # the last round's workgroups by CU: entry order on each CU and the duration of each
    hw = (st[:, 0].long() >> 8)
    cu = (xcc << 16) | (((hw >> 13) & 7) << 12) | (((hw >> 12) & 1) << 8) | ((hw >> 8) & 0xF)  # xcc, se, sh, cu
    t0 = st[:, 2].min()
    ent = (st[:, 2] - t0) / 100.0
    dur = (st[:, 4] - st[:, 2]) / 100.0
    print(f"last round: {int(cu.unique().numel())} CUs; workgroups per CU {sorted(collections.Counter(cu.tolist()).values())[:3]}..."
          f"{sorted(collections.Counter(cu.tolist()).values())[-3:]}")
    q = lambda v: " ".join(f"{x:6.1f}" for x in torch.quantile(v, torch.tensor([0.0, 0.1, 0.5, 0.9, 1.0], dtype=v.dtype)).tolist())
    print(f"entry us  q0/10/50/90/100: {q(ent)}")
    print(f"duration  q0/10/50/90/100: {q(dur)}")
    by_rank = collections.defaultdict(list)
    for c in cu.unique().tolist():
        idx = (cu == c).nonzero().flatten()
        order = idx[torch.argsort(ent[idx])]
        for k, i in enumerate(order.tolist()):
            by_rank[k].append((ent[i].item(), dur[i].item(), (ent[i] + dur[i]).item(), int(i)))
    for k in sorted(by_rank):
        v = by_rank[k]
        e_ = torch.tensor([x[0] for x in v]); d_ = torch.tensor([x[1] for x in v]); x_ = torch.tensor([x[2] for x in v])
        ids = torch.tensor([x[3] for x in v])
        print(f"k-th block on its CU, k={k}: n={len(v)} entry med {e_.median():6.1f} duration med {d_.median():6.1f} "
              f"(min {d_.min():6.1f} max {d_.max():6.1f}) exit med {x_.median():6.1f} max {x_.max():6.1f}; "
              f"blockIdx min/med/max {ids.min()}/{ids.median()}/{ids.max()}")


if __name__ == "__main__":
    main()
