#!/usr/bin/env python3
"""Interleaved A/B runs of bench.py variants on one GPU box (all variants once per round, so box
drift hits every variant alike).  Each variant = a name, environment overrides and bench.py
arguments; results (RTFx, ms/step, scan / GEMM launch us) print one line per run and go to
<out>.jsonl.  Usage (GPU box, repo root):
    python tools/ab_matrix.py <out> <rounds> 'name|VAR=v VAR2=w|--streams 1' ...
"""
import json
import os
import subprocess
import sys


def main():
    out, rounds = sys.argv[1], int(sys.argv[2])
    variants = []
    for spec in sys.argv[3:]:
        name, env, args = (spec.split("|") + ["", ""])[:3]
        variants.append((name, dict(kv.split("=", 1) for kv in env.split()), args.split()))
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    for r in range(rounds):
        for name, env, args in variants:
            e = dict(os.environ, **env)
            cmd = [sys.executable, "bench.py", "--no-cpu-baseline", "--no-scatter"] + args
            p = subprocess.run(cmd, env=e, capture_output=True, text=True, timeout=400)
            rec = dict(name=name, round=r, env=env, args=args, rc=p.returncode)
            if p.returncode == 0:
                d = json.loads(p.stdout.strip().splitlines()[-1])
                k = d["kernels"]
                rec.update(value=d["value"], ms=d["ms_per_step"],
                           scan_us=k["scan"]["avg_launch_us"] if k["scan"] else None,
                           gemm_us=k["gemm"]["avg_launch_us"], tokens_ok=d["rank0_tokens_match_reference"])
            else:
                rec["err"] = p.stderr[-2000:]
            print(json.dumps(rec), flush=True)
            with open(out + ".jsonl", "a") as f:
                f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
