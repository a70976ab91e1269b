#!/usr/bin/env python3
"""Throughput benchmark: VELOCITY-ASR inference, audio -> CTC tokens, on MI355X.

Workload (BASELINE.json configs[1]): the 6.17 M-parameter fp32 model, batch of 32 synthetic
10 s clips at 16 kHz per GPU.  One step = real-FFT |STFT|^2 + log-mel + full forward
(temporal binding, 8 SSM blocks, hierarchical global context, CTC head) + argmax + greedy
collapse, on audio already resident in HBM, replayed as one HIP graph.  Multi-GPU: one
process per GPU (torchrun), each rank transcribes its own 32 clips (utterance sharding, no
data-path collective; weak scaling); a barrier + synchronize brackets the K timed steps
and the max time over ranks is used.

Prints ONE JSON line (rank 0):
  value         = RTFx = audio seconds transcribed by all ranks / wall seconds
  roofline      = the dominant kernel family measured live with HIP events (eager replay of
                  the same steps on the launch stream) against the MI355X peak
  cpu_baseline  = the numpy restatement of the reference path (oracle/) on this host, a
                  bounded sample of the same workload (rank 0, N=1 only)
"""

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(REPO, "velocity-asr_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = json.load(open(os.path.join(REPO, "BASELINE.json")))["metric"]
SR = 16000
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
BF16_MFMA_PEAK_TFS = 2500.0  # dense bf16 MFMA (no sparsity)
F32_VALU_PEAK_TOPS = 78.6    # fp32 vector lane-operations/s (157.3 TFLOP/s with FMA = 2 flops)
VALU_OPS_PER_ELEM = 11       # reference tree scan, fp32 ops per state element (SURVEY §8 d)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_model(device):
    import velocity_asr as va
    from velocity_asr import synthetic as S
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    return m.to(device).eval()


def kernel_roofline(model, audio, steps, streams=1):
    """Per-launch times of the scan and GEMM families over `steps` eager steps (HIP events on
    each launch's own stream), run as the timed graphs run: `streams` utterance groups issued
    on concurrent streams, so the launches have the graph's shapes and the same overlap (and
    a rocprofv3 trace of this command sees one population per kernel)."""
    from velocity_asr import ops
    from velocity_asr.pipeline import audio_to_token_ids
    g = audio.shape[0] // streams
    sts = [torch.cuda.Stream(audio.device) for _ in range(streams)]
    main = torch.cuda.current_stream(audio.device)
    with ops.kernel_timer("ssm_scan", "gemm") as kt:
        for _ in range(steps):
            for i, st in enumerate(sts):
                st.wait_stream(main)
                with torch.cuda.stream(st):
                    audio_to_token_ids(model, audio[i * g:(i + 1) * g])
            for st in sts:
                main.wait_stream(st)
    rec = kt.summary()
    out = {}
    # selective scan of the 8 local blocks (N=64): bytes = B*L*(4*Di + 2*N)*4 per launch
    scans = [(dt, i) for dt, i in rec["ssm_scan"] if i["N"] == model.config.ssm_state_dim]
    if scans:
        i = scans[0][1]
        bytes_per = i["B"] * i["L"] * (4 * i["Di"] + 2 * i["N"]) * 4
        elems = i["B"] * i["L"] * i["Di"] * i["N"]
        t = float(np.mean([d for d, _ in scans]))
        out["scan"] = dict(t=t, bytes=bytes_per, elems=elems, launches=len(scans), per_step=len(scans) / steps,
                           total=sum(d for d, _ in scans) / steps, B=i["B"], Di=i["Di"])
    g = rec["gemm"]
    flops = [2.0 * i["M"] * i["N"] * i["K"] * i["batch"] for _, i in g]
    groups = {}
    for (d, i), f in zip(g, flops):
        k = (i["M"], i["N"], i["K"], i["batch"])
        groups.setdefault(k, []).append((d, f))
    top = max(groups.items(), key=lambda kv: sum(d for d, _ in kv[1]))
    out["gemm"] = dict(t=float(np.mean([d for d, _ in g])), flops=float(np.mean(flops)), launches=len(g),
                       per_step=len(g) / steps, total=sum(d for d, _ in g) / steps,
                       tflops=sum(flops) / max(sum(d for d, _ in g), 1e-12) / 1e12,
                       top_shape="M=%d N=%d K=%d batch=%d" % top[0], top_t=float(np.mean([d for d, _ in top[1]])),
                       top_flops=top[1][0][1], top_total=sum(d for d, _ in top[1]) / steps)
    return out


def cpu_baseline(seconds_target=12.0):
    """Oracle (numpy port of the reference path) on 10 s clips until ~seconds_target of work."""
    from oracle import velocity_ref as R
    from velocity_asr import synthetic as S
    try:
        from threadpoolctl import threadpool_info
        threads = max([d.get("num_threads", 1) for d in threadpool_info()] or [1])
    except Exception:  # pragma: no cover
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    W = S.make_weights(None, seed=0)
    cfg = dict(S.DEFAULT_CONFIG)
    clips, t0 = 0, time.perf_counter()
    while True:
        a = S.make_audio(1, 10 * SR, seed=1234 + clips)
        R.ctc_greedy_decode(R.forward(W, R.compute_mel_spectrogram(a), cfg))
        clips += 1
        el = time.perf_counter() - t0
        if el >= seconds_target or clips >= 32:
            break
    return dict(value=round(clips * 10.0 / el, 3), unit="audio-sec/sec (RTFx)", cores=int(threads), kind="port",
                sample=f"{clips} x 10 s clips, batch 1, mel+forward+greedy, oracle/velocity_ref.py "
                       f"(numpy, BLAS threads={threads}), {el:.1f} s wall")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32, help="clips per GPU")
    ap.add_argument("--seconds", type=float, default=10.0, help="clip length")
    ap.add_argument("--eager", action="store_true", help="time eager launches instead of the HIP graph")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--roofline-steps", type=int, default=3)
    ap.add_argument("--streams", type=int, default=2,
                    help="utterance groups replayed as separate HIP graphs on concurrent streams (the scan of one "
                         "group overlaps the GEMMs of the other; results are bitwise those of one graph)")
    ap.add_argument("--int8", action="store_true",
                    help="BASELINE configs[4]: INT8 fake-quant model (prepare_model_for_qat + activation calibration)")
    ap.add_argument("--bf16", action="store_true",
                    help="BASELINE configs[2] per-GPU shape: the model as bf16 (bf16 weights / MFMA operands)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from velocity_asr import synthetic as S
    from velocity_asr.pipeline import GraphedTranscriber, audio_to_token_ids

    model = build_model(dev)
    if args.bf16:
        model = model.to(torch.bfloat16)
    if args.int8:
        from velocity_asr import compute_mel_spectrogram
        from velocity_asr import quantize as Q
        model = Q.prepare_model_for_qat(model).to(dev).eval()
        calib = torch.from_numpy(S.make_audio(2, 48000, seed=71)).to(dev)
        Q.calibrate_from_activations(model, compute_mel_spectrogram(calib))
    S_len = int(args.seconds * SR)
    B = args.batch
    audio = torch.from_numpy(S.make_audio(B, S_len, seed=1234 + rank)).to(dev)  # resident in HBM

    if args.eager:
        def step():
            return audio_to_token_ids(model, audio)
    else:
        tr = GraphedTranscriber(model, B, S_len, dev, streams=args.streams)
        tr.audio.copy_(audio)
        step = tr.step

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # token checksum over all ranks (tiny gather, outside the timed region); the timed graph's
    # own output must equal an eager pass over the same audio
    toks, lens = audio_to_token_ids(model, audio)
    graph_match = True
    if not args.eager:
        from velocity_asr.pipeline import token_lists
        gt, gl = tr.collect()
        graph_match = token_lists(gt, gl) == token_lists(toks, lens)
    valid = torch.arange(toks.shape[1], device=dev)[None, :] < lens[:, None]
    csum = torch.tensor([float(lens.sum().item()), float(toks.long().masked_fill(~valid, 0).sum().item())],
                        device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(csum)

    rf = kernel_roofline(model, audio, args.roofline_steps, 1 if args.eager else args.streams)
    if world > 1:
        dist.barrier()
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    audio_sec = world * B * args.seconds * args.steps
    frames = world * B * (S_len // 160 + 1) * args.steps
    ms_per_step = elapsed / args.steps * 1e3
    sc, gm = rf.get("scan"), rf["gemm"]
    # dominant kernel = the single kernel (same code, same shape) with the largest time per step
    if sc and sc["total"] >= gm["top_total"]:
        ach = sc["bytes"] / sc["t"] / 1e9
        roof = dict(bound="hbm", kernel="vasr ssm_scan (tree scan + gate, 8 local blocks, B*L*(4*Di+2*N)*4 B/launch)",
                    achieved=round(ach, 1), peak=HBM_PEAK_GBS, unit="GB/s", frac=round(ach / HBM_PEAK_GBS, 4),
                    traffic=None, avg_launch_us=round(sc["t"] * 1e6, 2))
        # the scan is VALU-bound: the same launch against the fp32 vector roof, at the
        # reference tree's ~11 fp32 operations per state element (SURVEY §8 d), FMA counted once
        tops = sc["elems"] * VALU_OPS_PER_ELEM / sc["t"] / 1e12
        roof["valu"] = dict(ops_per_element=VALU_OPS_PER_ELEM, achieved=round(tops, 2), peak=F32_VALU_PEAK_TOPS,
                            unit="T lane-ops/s", frac=round(tops / F32_VALU_PEAK_TOPS, 4))
        key = "ssm_scan"
    else:
        # split-bf16 GEMM: six bf16 MFMA products per fp32 multiply-add, against the dense bf16 roof
        ach = 6 * gm["top_flops"] / gm["top_t"] / 1e12
        roof = dict(bound="mfma", kernel=f"vasr gemm_x3 {gm['top_shape']} (6 bf16 products)", achieved=round(ach, 2),
                    peak=BF16_MFMA_PEAK_TFS, unit="TFLOP/s", frac=round(ach / BF16_MFMA_PEAK_TFS, 4), traffic=None,
                    avg_launch_us=round(gm["top_t"] * 1e6, 2))
        key = "gemm_x3"
    pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            t = json.load(open(pmc)).get(key)
            if isinstance(t, dict) and sc:  # by launch grid: B x Di/16 blocks of 256 threads
                t = t.get(str(sc["B"] * (sc["Di"] // 16) * 256))
            roof["traffic"] = t
        except Exception:
            pass
    line = {
        "metric": METRIC,
        "value": round(audio_sec / elapsed, 2),
        "unit": "audio-sec/sec (RTFx)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if args.bf16 else "f32",
        "data": "synthetic: N(0, 0.1) 16 kHz clips; seeded random-init weights (velocity_asr.synthetic)",
        "config": {"workload": f"{B} x {args.seconds:g} s clips per GPU, audio->mel->forward->CTC greedy tokens "
                               f"(BASELINE configs[{4 if args.int8 else 2 if args.bf16 else 1}]"
                               f"{', INT8 fake-quant' if args.int8 else ''}"
                               f"{f', HIP graph x{args.streams} streams' if not args.eager else ', eager'})",
                   "global_batch": world * B, "clip_seconds": args.seconds, "parallelism": f"utterance-shard x{world}"},
        "frames_per_sec": round(frames / elapsed, 1),
        "roofline": roof,
        "kernels": {
            "scan": None if not sc else dict(avg_launch_us=round(sc["t"] * 1e6, 2), launches_per_step=sc["per_step"],
                                             ms_per_step=round(sc["total"] * 1e3, 3),
                                             hbm_gbs=round(sc["bytes"] / sc["t"] / 1e9, 1),
                                             gelem_per_s=round(sc["elems"] / sc["t"] / 1e9, 1)),
            "gemm": dict(avg_launch_us=round(gm["t"] * 1e6, 2), launches_per_step=gm["per_step"],
                         ms_per_step=round(gm["total"] * 1e3, 3), tflops=round(gm["tflops"], 2)),
        },
        "token_checksum": [int(csum[0].item()), int(csum[1].item())],
        "graph_tokens_match_eager": graph_match,
    }
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline()
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
