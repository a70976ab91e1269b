#!/usr/bin/env python3
"""Summarise tools/pmc_mfma.sh runs (gpurun_out/mfma_<tag>_<M>) into profiles/.

Per GEMM shape (dispatch order from tools/gemm_pmc.py: 1 warm-up + REPS counted launches):
  dur_us            mean kernel duration from the un-profiled --kernel-trace pass
  mops_flops        SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 = bf16 MFMA flops the kernel issued
  mfma_tflops       mops_flops / dur, against the dense bf16 peak (2.5 PF): mfma_frac
  busy_per_simd     SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs (cycles the MFMA pipe was busy)
  mfma_busy_frac    busy_per_simd / (dur x 2.4 GHz): MFMA-pipe occupancy at the peak clock
                    (the chip runs below 2.4 GHz under MFMA load, MI355X_MICROARCH.md 'DVFS',
                    so this reads as a lower bound)
  f32eq_tflops      2*M*N*K / dur against the f32-MFMA peak (157.3 TF)
Writes profiles/pmc_mfma.json ({"M,N,K": {...}}, read by bench.py) and
profiles/<tag>_gemm_mfma.md.  Usage: python tools/summarize_mfma.py <tag> <M> [<M> ...]
"""
import collections
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLOCK = 2.4e9
SIMDS = 1024
PEAK_BF16 = 2500e12
PEAK_F32 = 157.3e12


FAMILIES = ("gemm_x3_kernel", "gemm_rows_kernel", "ssm_tail_gated_kernel", "ssm_tail_kernel")


def family_rows(path):
    """{kernel family: [rows sorted by dispatch]} of the counted kernel families."""
    fam = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        for f in FAMILIES:
            if f in r["Kernel_Name"]:
                fam[f].append(r)
    return fam


def main(tag, Ms):
    out_json = os.path.join(REPO, "profiles", "pmc_mfma.json")
    table = json.load(open(out_json)) if os.path.exists(out_json) else {}
    md = [f"# MFMA utilisation of the split-bf16 GEMMs ({tag})", "",
          "rocprofv3 counters over `tools/gemm_pmc.py` (isolated launches, random operands), durations from the "
          "un-profiled kernel-trace pass of the same script; `tools/pmc_mfma.sh` + `tools/summarize_mfma.py`.", "",
          "| M | shape | kernel | N | K | dur µs | MFMA flops counted / expected | MFMA TF/s | of 2.5 PF | busy cyc/SIMD | "
          "busy frac @2.4 GHz | fp32-eq TF/s | of 157.3 TF |", "|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for M in Ms:
        src = os.path.join(REPO, "gpurun_out", f"mfma_{tag}_{M}")
        order = json.load(open(os.path.join(src, "order.json")))
        trace = family_rows(os.path.join(src, "trace", "run_kernel_trace.csv"))
        pmc = family_rows(os.path.join(src, "pmc", "run_counter_collection.csv"))
        durs = {f: [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"]))] for f, rows in trace.items()}
        disp = {}
        for f, rows in pmc.items():
            cnt = collections.defaultdict(dict)
            for r in rows:
                d = cnt[int(r["Dispatch_Id"])]
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            disp[f] = [cnt[k] for k in sorted(cnt)]
        seen = collections.Counter()
        for sh in order:
            f = sh.get("kernel", "gemm_x3_kernel")
            per = sh["reps"] + 1
            i = seen[f]
            seen[f] += 1
            sl = slice(i * per + 1, (i + 1) * per)  # drop the warm-up launch
            dur = sum(durs[f][sl]) / (per - 1) * 1e-9
            c = disp[f][sl]
            assert len(c) == per - 1, (sh["name"], len(c))
            mops = sum(x["SQ_INSTS_VALU_MFMA_MOPS_BF16"] for x in c) / len(c) * 512
            busy = sum(x["SQ_VALU_MFMA_BUSY_CYCLES"] for x in c) / len(c) / SIMDS
            expect = sh["flops"] * sh["bf16_products"]
            ent = dict(name=sh["name"], kernel=f, dur_us=round(dur * 1e6, 2), mops_flops=mops, expected_flops=expect,
                       mfma_tflops=round(mops / dur / 1e12, 1), mfma_frac=round(mops / dur / PEAK_BF16, 4),
                       busy_per_simd=round(busy), mfma_busy_frac=round(busy / (dur * CLOCK), 4),
                       f32eq_tflops=round(sh["flops"] / dur / 1e12, 2), f32eq_frac=round(sh["flops"] / dur / PEAK_F32, 4))
            key = ("%d,%d,%d" % (sh["M"], sh["N"], sh["K"]) if f.startswith("gemm_")
                   else ("tailg,%d" if "gated" in f else "tail,%d") % sh["M"])
            table[key] = ent
            md.append(f"| {sh['M']} | {sh['name']} | {f} | {sh['N']} | {sh['K']} | {ent['dur_us']} | {mops / expect:.3f} | "
                      f"{ent['mfma_tflops']} | {ent['mfma_frac']:.3f} | {ent['busy_per_simd']} | "
                      f"{ent['mfma_busy_frac']:.3f} | {ent['f32eq_tflops']} | {ent['f32eq_frac']:.3f} |")
    json.dump(table, open(out_json, "w"), indent=1, sort_keys=True)
    open(os.path.join(REPO, "profiles", f"{tag}_gemm_mfma.md"), "w").write("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main(sys.argv[1], [int(m) for m in sys.argv[2:]] or [8016])
