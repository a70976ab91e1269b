#!/usr/bin/env python3
"""Diagnostic (CPU side): code objects of stft.hip's SLP-vectorised kernel with chosen packed-fp32
instructions rewritten as their two scalar halves, for tools/diag/interference_seq.py's module victim
(VICTIM_HSACO).  Which packed form, replaced alone, removes the perturbation beside the mel -> conv
GEMM sequence of another stream?

    python tools/diag/stft_surgery.py OUTDIR          # writes OUTDIR/stft_<mode>.hsaco + a report

Modes (each a whole-kernel rewrite of the same SLP build, same registers, same schedule otherwise):
  none    the SLP build as compiled (the pipeline check: must still fail)
  all     every v_pk_{add,mul,fma}_f32 and v_pk_mov_b32 -> two VOP3 scalar instructions
  opsel   only the packed ops whose low half reads a high dword (an op_sel bit set: re/im swaps)
  neg     only the packed ops with neg_lo / neg_hi modifiers (and no op_sel bit)
  plain   only the packed ops with neither (no op_sel bit, no neg)
  opsel_mov / opsel_swap / opsel_bcast   the op_sel class split: v_pk_mov_b32; a source with
          op_sel 1 / op_sel_hi 0 (its dwords swapped); a source with op_sel 1 / op_sel_hi 1 (its high
          dword in both halves)
A packed op D = op(A, B[, C]) computes D.lo from each source's dword op_sel[i] and D.hi from dword
op_sel_hi[i] (defaults 0 / 1), with neg_lo / neg_hi negating a source in that half; the rewrite
emits the half whose destination the other half does not read first.
"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(REPO, "velocity-asr_amd")
LLVM = "/opt/rocm/lib/llvm/bin"
HIPCC = "/opt/rocm/bin/hipcc"
SCALAR = {"v_pk_add_f32": "v_add_f32_e64", "v_pk_mul_f32": "v_mul_f32_e64", "v_pk_fma_f32": "v_fma_f32",
          "v_pk_mov_b32": "v_mov_b32_e32"}


def _mods(text, key, n, default):
    m = re.search(key + r":\[([01,]+)\]", text)
    v = [int(x) for x in m.group(1).split(",")] if m else []
    return v + [default] * (n - len(v))


def _half(op, half):
    """The 32-bit register / constant a 64-bit packed operand supplies for dword `half`."""
    m = re.fullmatch(r"([vs])\[(\d+):(\d+)\]", op)
    if m:
        return f"{m.group(1)}{int(m.group(2)) + half}"
    return op  # inline constant or literal: the same 32-bit value in either half


def split(line):
    """[scalar instruction, ...] equivalent to one packed instruction line, or None."""
    body = line.strip().split(";")[0].strip()
    op = body.split()[0]
    if op not in SCALAR:
        return None
    rest = body[len(op):].strip()
    mods_at = min([rest.find(k) for k in ("op_sel", "neg_lo", "neg_hi") if rest.find(k) >= 0] or [len(rest)])
    operands = [o.strip() for o in rest[:mods_at].split(",")]
    dst, srcs = operands[0], operands[1:]
    n = len(srcs)
    sel = _mods(rest, "op_sel", n, 0)
    selhi = _mods(rest, "op_sel_hi", n, 1)
    nlo = _mods(rest, "neg_lo", n, 0)
    nhi = _mods(rest, "neg_hi", n, 0)
    if op == "v_pk_mov_b32":  # D.lo = src0[op_sel[0]], D.hi = src1[op_sel[1]]
        lo_src, hi_src = [_half(srcs[0], sel[0])], [_half(srcs[1], sel[1])]
        lo = f"v_mov_b32_e32 {_half(dst, 0)}, {lo_src[0]}"
        hi = f"v_mov_b32_e32 {_half(dst, 1)}, {hi_src[0]}"
    else:
        def emit(h, selv, neg):
            args = [("-" if neg[i] else "") + _half(s, selv[i]) for i, s in enumerate(srcs)]
            return f"{SCALAR[op]} {_half(dst, h)}, " + ", ".join(args), [_half(s, selv[i]) for i, s in enumerate(srcs)]
        lo, lo_src = emit(0, sel, nlo)
        hi, hi_src = emit(1, selhi, nhi)
    d0, d1 = _half(dst, 0), _half(dst, 1)
    if d0 in hi_src and d1 in lo_src:
        if lo.split(None, 2)[2] == hi.split(None, 2)[2]:  # both halves the same value: compute once, copy
            return [lo, f"v_mov_b32_e32 {d1}, {d0}"]
        raise ValueError(f"cyclic halves, needs a temporary: {line.strip()}")
    return [hi, lo] if d0 in hi_src else [lo, hi]


def classify(line):
    body = line.strip().split(";")[0]
    op = body.split()[0] if body.split() else ""
    if op not in SCALAR:
        return None
    has_sel = re.search(r"op_sel:\[[01,]*1", body) is not None
    has_neg = "neg_lo" in body or "neg_hi" in body
    return "opsel" if has_sel else "neg" if has_neg else "plain"


def opsel_kind(line):
    """The op_sel sub-class of a packed op with an op_sel bit set: 'mov' (v_pk_mov_b32), 'swap'
    (a source whose low half reads its high dword and whose high half reads its low dword), 'bcast'
    (a source read as its high dword in both halves)."""
    body = line.strip().split(";")[0]
    op = body.split()[0]
    if op == "v_pk_mov_b32":
        return "mov"
    n = body.count(",")  # sources = commas before the modifiers (dst, s0, s1[, s2])
    sel, selhi = _mods(body, "op_sel", 3, 0), _mods(body, "op_sel_hi", 3, 1)
    return "swap" if any(sel[i] == 1 and selhi[i] == 0 for i in range(3)) else "bcast"


SUBMODES = ("opsel_mov", "opsel_swap", "opsel_bcast")


def rewrite(asm_lines, mode, kernel):
    out, n, inside = [], 0, False
    for line in asm_lines:
        if line.startswith(kernel + ":"):
            inside = True
        elif inside and line.startswith(".Lfunc_end"):
            inside = False
        c = classify(line) if inside else None
        if c == "opsel" and mode in SUBMODES:
            c = "opsel_" + opsel_kind(line)
        if c is not None and (mode == "all" or mode == c):
            out += ["\t" + s + "\n" for s in split(line)]
            n += 1
        else:
            out.append(line)
    return out, n


def main(outdir):
    os.makedirs(outdir, exist_ok=True)
    asm = os.path.join(outdir, "stft_slp.s")
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-I../include", "-munsafe-fp-atomics",
                    "-fslp-vectorize", "--cuda-device-only", "-S", "csrc/stft.hip", "-o", asm], cwd=PKG, check=True,
                   capture_output=True)
    lines = open(asm).readlines()
    kernel = next(ln.split(":")[0] for ln in lines if re.match(r"^_Z\w*stft_power_400_kernel\w*:", ln))
    report = [f"kernel {kernel}"]
    for mode in ("none", "all", "opsel", "neg", "plain") + SUBMODES:
        new, n = rewrite(lines, mode, kernel)
        s = os.path.join(outdir, f"stft_{mode}.s")
        open(s, "w").writelines(new)
        o, co = s[:-2] + ".o", s[:-2] + ".hsaco"
        subprocess.run([os.path.join(LLVM, "clang"), "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                        "-mcpu=gfx950", "-c", s, "-o", o], check=True)
        subprocess.run([os.path.join(LLVM, "ld.lld"), "-shared", o, "-o", co], check=True)
        dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co], check=True,
                             capture_output=True, text=True).stdout
        left = sum(1 for ln in dis.splitlines() if re.search(r"\bv_pk_(add|mul|fma)_f32|\bv_pk_mov_b32", ln))
        report.append(f"{mode:6s}: {n:3d} packed instructions rewritten, {left:3d} left -> {co}")
    open(os.path.join(outdir, "report.txt"), "w").write("\n".join(report) + "\n")
    print("\n".join(report))
    print("kernel_symbol", kernel)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "tools", "_variants", "surgery"))
