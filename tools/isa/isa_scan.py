#!/usr/bin/env python3
"""Scan the gfx950 machine code shipped in libvasr_hip.so for instruction sequences.

The library's `.hip_fatbin` section holds one clang offload bundle per translation unit; each
bundle's gfx950 entry is an AMDGPU code object, disassembled here with the ROCm llvm-objdump.

The form it guards against: a packed-fp32 VOP3P arithmetic
instruction (`v_pk_{add,mul,fma}_f32`) with a SWAPPED source -- op_sel[i] = 1 and op_sel_hi[i] = 0,
so the low half reads the source pair's high dword and the high half its low dword (the compiler's
re/im swap of complex arithmetic, or x + y of a pair's halves).  stft.hip built with SLP
vectorisation returned wrong |STFT|^2 values for a (half-)wave now and then when MFMA kernels of
another stream shared the SIMD (18/400 launches); rewriting only its 12 swapped-source instructions
as scalar pairs removed that (0/400), while rewriting every other packed form (SGPR-pair sources,
high-dword broadcasts, v_pk_mov_b32 with op_sel, neg modifiers, plain) left it (18-19/400):
tools/diag/stft_surgery.py, tools/runs/r05e.sh / r05f.sh, profiles/r05e/, r05f/.

    python tools/isa/isa_scan.py [lib.so]          # report per kernel
"""
import os
import re
import shutil
import struct
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB = os.path.join(REPO, "velocity-asr_amd", "velocity_asr", "lib", "libvasr_hip.so")
OBJDUMP_CANDIDATES = ("/opt/rocm/lib/llvm/bin/llvm-objdump", "/opt/rocm/llvm/bin/llvm-objdump")
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "gfx950"


def objdump():
    for p in OBJDUMP_CANDIDATES:
        if os.path.exists(p):
            return p
    p = shutil.which("llvm-objdump")
    if p:
        return p
    raise FileNotFoundError("llvm-objdump not found")


def elf_section(path, name):
    """Bytes of section `name` of a 64-bit little-endian ELF file."""
    d = open(path, "rb").read()
    if d[:4] != b"\x7fELF" or d[4] != 2 or d[5] != 1:
        raise ValueError(f"{path}: not a 64-bit little-endian ELF")
    shoff = struct.unpack_from("<Q", d, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", d, 0x3A)
    def sh(i):
        return struct.unpack_from("<IIQQQQIIQQ", d, shoff + i * shentsize)
    stroff = sh(shstrndx)[4]
    for i in range(shnum):
        nm, _typ, _fl, _addr, off, size = sh(i)[:6]
        end = d.index(b"\0", stroff + nm)
        if d[stroff + nm:end].decode() == name:
            return d[off:off + size]
    raise KeyError(f"{path}: no section {name}")


def code_objects(lib=LIB):
    """The gfx950 code objects of every offload bundle in the library's .hip_fatbin section."""
    fat = elf_section(lib, ".hip_fatbin")
    out = []
    pos = fat.find(BUNDLE_MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", fat, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if triple.endswith(TARGET) and size:
                out.append(fat[pos + off:pos + off + size])
        pos = fat.find(BUNDLE_MAGIC, pos + 1)
    return out


def disassemble(co_bytes):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co_bytes)
        f.flush()
        r = subprocess.run([objdump(), "-d", "--no-show-raw-insn", "--demangle", f.name], capture_output=True,
                           text=True, check=True)
    return r.stdout


def kernels(text):
    """{symbol: [instruction text, ...]} from llvm-objdump output."""
    ks, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.*)>:$", line)
        if m:
            cur = m.group(1)
            ks[cur] = []
            continue
        s = line.strip()
        if cur is None or not s or s.startswith(";"):
            continue
        s = s.split("//")[0].strip()
        if s:
            ks[cur].append(s)
    return ks


def library_kernels(lib=LIB):
    ks = {}
    for co in code_objects(lib):
        for name, ins in kernels(disassemble(co)).items():
            if ins:
                ks[name] = ins
    return ks


def _operands(ins):
    parts = ins.split(None, 1)
    if len(parts) < 2:
        return []
    return [o.strip().split()[0] for o in parts[1].split(",") if o.strip()]


def _opsel(ins, key, n, default):
    m = re.search(key + r":\[([01,]+)\]", ins)
    if not m:
        return [default] * n
    v = [int(x) for x in m.group(1).split(",")]
    return v + [default] * (n - len(v))


PACKED_F32 = re.compile(r"v_pk_(add|mul|fma)_f32\b")


def swapped_sources(ins):
    """Indices of the sources whose dwords a packed-fp32 instruction reads swapped."""
    if not PACKED_F32.match(ins):
        return []
    n = len(_operands(ins)) - 1
    sel, selhi = _opsel(ins, "op_sel", n, 0), _opsel(ins, "op_sel_hi", n, 1)
    return [i for i in range(n) if sel[i] == 1 and selhi[i] == 0]


def pk_swapped(ins_list):
    """[(index, instruction)] of the packed-fp32 instructions with a swapped source."""
    return [(i, s) for i, s in enumerate(ins_list) if swapped_sources(s)]


def main(argv):
    lib = argv[1] if len(argv) > 1 else LIB
    ks = library_kernels(lib)
    total = 0
    for name in sorted(ks):
        ins = ks[name]
        npk = sum(1 for s in ins if PACKED_F32.match(s))
        hits = pk_swapped(ins)
        total += len(hits)
        if npk or hits:
            print(f"{len(ins):6d} instr  {npk:5d} v_pk_*_f32  {len(hits):3d} with a swapped source  {name[:110]}")
        for i, s in hits[:4]:
            print(f"      [{i}] {s}")
    print(f"{len(ks)} kernels, {total} packed-fp32 instructions with a swapped source")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
