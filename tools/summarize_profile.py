#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (gpurun_out/prof_<tag>) into profiles/<tag>_*.

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_summary.md         per-kernel table: calls, avg us, share, HBM bytes/launch
  profiles/pmc_traffic.json         per-kernel-family HBM bytes per launch, used by bench.py

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE come from separate
--pmc passes (KiB units); FETCH_SIZE is doubled on gfx950 (it tallies 128-B requests at
64 B; calibrated here on layer_norm_kernel, whose 12.3 MB read shows as 6.04 MB), WRITE_SIZE
is taken as is (it matches the scan's 24.6 MB output exactly).
"""

import collections
import csv
import json
import os
import re
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    n = name.replace("void ", "").replace("vasr::(anonymous namespace)::", "")
    return n.split("(")[0]


def family(name):
    n = short(name)
    if re.search(r"(^|::)ssm_scan_kernel<64, [02],", n):  # tree modes, either lane layout
        return "ssm_scan"
    if n.startswith("gemm_f32_kernel"):
        return "gemm_f32"
    return n.split("<")[0]


def pmc(path, counter):
    agg = collections.defaultdict(list)
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[(short(r["Kernel_Name"]), r["Grid_Size"])].append(float(r["Counter_Value"]))
    return agg


def main(tag):
    src = os.path.join(REPO, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(REPO, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    fetch = pmc(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = pmc(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    per_kernel = {}  # (kernel, grid) -> (read bytes, write bytes, launches)
    for key in set(fetch) | set(write):
        f = fetch.get(key, [0.0])
        w = write.get(key, [0.0])
        per_kernel[key] = (2 * 1024 * sum(f) / len(f), 1024 * sum(w) / len(w), max(len(f), len(w)))
    lines = [f"# rocprofv3 summary, run {tag}", "",
             "| kernel | calls | avg us | share % | HBM read MB/launch | HBM write MB/launch |",
             "|---|---|---|---|---|---|"]
    traffic = {}
    for r in rows:
        n = short(r["Name"])
        # the launch population (grid size) with the most launches: the timed graphs' shape
        cands = sorted(((v[2], g, v) for (k, g), v in per_kernel.items() if k == n), reverse=True)
        rd = cands[0][2][0] if cands else None
        wr = cands[0][2][1] if cands else None
        lines.append(f"| `{n[:70]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                     f"{float(r['Percentage']):.2f} | {'' if rd is None else f'{rd / 1e6:.1f}'} | "
                     f"{'' if wr is None else f'{wr / 1e6:.1f}'} |")
        fam = family(r["Name"])
        if fam in ("ssm_scan",) and rd is not None:
            # "grid size @ L" -> bytes, merged over the family's instantiations (chunk lengths,
            # layouts); tools/profile.sh profiles the C2 bench, L = SCAN_L (501)
            traffic.setdefault(fam, {}).update({f"{g}@{SCAN_L}": int(v[0] + v[1]) for _, g, v in cands})
    lines += isolated_runs(os.path.join(src, "trace", "run_kernel_trace.csv"),
                           os.path.join(src, "bench_trace.json"))
    with open(os.path.join(dst, f"{tag}_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    with open(os.path.join(dst, "pmc_traffic.json"), "w") as f:
        json.dump(dict(run=tag, unit="bytes per launch (FETCH_SIZE*2 + WRITE_SIZE), by launch grid size (threads) "
                                     "@ time steps", **traffic), f, indent=1)
    print("\n".join(lines[:14]))


def isolated_runs(trace, bench_json, reps=20):
    """bench.py's isolated_times(): `reps` back-to-back launches of one kernel (after 3 warm-up
    launches), timed by one HIP event pair.  Found in the kernel trace as runs of >= reps + 3
    consecutive dispatches of one kernel; the last `reps` give the average kernel duration and
    the span / reps (the event pair's quantity: durations plus dispatch gaps), to set beside the
    avg_launch_us the profiled bench line printed."""
    if not os.path.exists(trace):
        return []
    ks = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    runs, i = [], 0
    while i < len(ks):
        j = i
        while j + 1 < len(ks) and ks[j + 1]["Kernel_Name"] == ks[i]["Kernel_Name"]:
            j += 1
        if j - i + 1 >= reps + 3:
            sel = ks[j + 1 - reps:j + 1]
            dur = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sel) / reps / 1e3
            span = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / reps / 1e3
            runs.append((short(ks[i]["Kernel_Name"]), j - i + 1, dur, span))
        i = j + 1
    out = ["", f"## Isolated back-to-back runs (bench.py isolated_times: 3 warm-up + {reps} timed launches)", "",
           "| kernel | run length | avg kernel us (last 20) | span / 20 us |", "|---|---|---|---|"]
    out += [f"| `{n[:70]}` | {ln} | {d:.2f} | {sp:.2f} |" for n, ln, d, sp in runs]
    if os.path.exists(bench_json):
        try:
            r = json.load(open(bench_json))["roofline"]
            out += ["", f"The profiled bench line (bench_trace.json, same process): avg_launch_us {r['avg_launch_us']} "
                        f"({r['kernel'].split(' (')[0]}), gemm_avg_launch_us {r['gemm_avg_launch_us']} "
                        f"({r['gemm_kernel']})."]
        except (ValueError, KeyError):
            pass
    return out


SCAN_L = int(os.environ.get("SCAN_L", "501"))  # time steps of the profiled bench's scans

if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
