#!/usr/bin/env python3
"""Per-launch means of the SQ counters a tools/pmc_kernel.sh run collected for one kernel.

    python tools/pmc_means.py gpurun_out/pmc_<tag> <kernel-name substring> [steps]

Prints every counter's mean over the kernel's dispatches and, with `steps` (time steps each
wave walks, e.g. L = 501 for the scan), the per-wave-step instruction counts and the issue
fractions (SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES, SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES).
"""
import collections
import csv
import glob
import os
import sys


def main():
    root, pat = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    sums, counts = collections.defaultdict(float), collections.defaultdict(set)
    for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if pat not in r["Kernel_Name"]:
                continue
            c = r["Counter_Name"]
            sums[c] += float(r["Counter_Value"])
            counts[c].add((f, r["Dispatch_Id"]))
    m = {c: sums[c] / len(counts[c]) for c in sums}
    for c in sorted(m):
        print(f"{c} {m[c]:.4g}")
    if steps and m.get("SQ_WAVES"):
        ws = m["SQ_WAVES"] * steps
        print(f"VALU per wave-step {m.get('SQ_INSTS_VALU', 0) / ws:.2f} LDS per wave-step "
              f"{m.get('SQ_INSTS_LDS', 0) / ws:.2f} SALU per wave-step {m.get('SQ_INSTS_SALU', 0) / ws:.2f}")
    if m.get("SQ_WAVE_CYCLES"):
        wc = m["SQ_WAVE_CYCLES"]
        print(f"ACTIVE_INST_ANY/WAVE_CYCLES {m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f} "
              f"WAIT_INST_ANY/WAVE_CYCLES {m.get('SQ_WAIT_INST_ANY', 0) / wc:.3f} "
              f"WAIT_ANY/WAVE_CYCLES {m.get('SQ_WAIT_ANY', 0) / wc:.3f} "
              f"ACTIVE_INST_VALU/WAVE_CYCLES {m.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f}")
    if m.get("GRBM_GUI_ACTIVE") and m.get("SQ_ACTIVE_INST_VALU"):
        # GRBM_GUI_ACTIVE sums the 8 XCDs' clocks; SQ_ACTIVE_INST_* count quad-cycles over all waves
        cyc = m["GRBM_GUI_ACTIVE"] / 8
        print(f"kernel cycles {cyc:.4g}; SIMD VALU busy (ACTIVE_INST_VALU x 4 / (1024 SIMDs x cycles)) "
              f"{4 * m['SQ_ACTIVE_INST_VALU'] / (1024 * cyc):.3f}; SIMD issue busy (ACTIVE_INST_ANY x 4 / "
              f"(1024 x cycles)) {4 * m.get('SQ_ACTIVE_INST_ANY', 0) / (1024 * cyc):.3f}")


if __name__ == "__main__":
    main()
