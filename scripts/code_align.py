"""Where a kernel's 8-byte (VOP3 / VOP3P) VALU instructions sit relative to 8-byte boundaries.

The VALU-bound kernels here run 10-15 % faster when nearly all of their 8-byte instructions sit
at addresses 4 mod 8 than when they sit at 0 mod 8 (same code, moved by 4 bytes: key hashing
10.3 vs 11.8 ms, the leaf kernel 13.4 vs 14.7 ms at 100M; profiles/r8d_*, r8k_*).  The
assembler places instructions back to back, so which case a kernel gets follows from the
size of everything before it; this tool reads it off a built object.

  python scripts/code_align.py build/libkhst_khst.o [kernel-name-substring ...]

Measurement / build-check tool (scripts/, not the library)."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def disassemble(obj):
    """objdump text of every gfx950 code object in a host object's (or shared library's)
    .hip_fatbin: one offload bundle per compilation unit, back to back."""
    out = []
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fb")
        subprocess.check_call(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fb])
        data = open(fb, "rb").read()
        starts = [k for k in range(len(data)) if data.startswith(MAGIC, k)] if data.count(MAGIC) else []
        for n, a in enumerate(starts):
            b = starts[n + 1] if n + 1 < len(starts) else len(data)
            part, co = os.path.join(d, f"b{n}"), os.path.join(d, f"co{n}")
            open(part, "wb").write(data[a:b])
            subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + part,
                                   "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co])
            out.append(subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], capture_output=True, text=True,
                                      check=True).stdout)
    return "\n".join(out)


def kernels(txt):
    """{symbol: [(address, text), ...]}"""
    out = {}
    heads = list(re.finditer(r"^([0-9a-f]{16}) <(_Z\w+)>:", txt, re.M))
    for k, h in enumerate(heads):
        end = heads[k + 1].start() if k + 1 < len(heads) else len(txt)
        body = txt[h.end():end]
        out[h.group(2)] = [(int(a, 16), t.strip()) for t, a in re.findall(r"\t([^\n]*?)\s*//\s*([0-9A-F]{12}):", body)]
    return out


def stats(ins):
    v8 = v8m = 0
    for k in range(len(ins) - 1):
        a, t = ins[k]
        if ins[k + 1][0] - a == 8 and t.startswith("v_"):
            v8 += 1
            v8m += a % 8 == 4
    return v8, v8m


def main():
    obj, subs = sys.argv[1], sys.argv[2:]
    for sym, ins in sorted(kernels(disassemble(obj)).items()):
        if subs and not any(s in sym for s in subs):
            continue
        v8, v8m = stats(ins)
        if v8 >= 200:
            print(f"{sym[:60]:60s} valu8B {v8:6d}  at 4 mod 8: {v8m / v8:5.2f}")


if __name__ == "__main__":
    main()


def loops(ins, min_len=2048):
    """(head, tail, valu8B, at 4 mod 8) of the back-edges spanning >= min_len bytes"""
    lab = {}
    out = []
    addrs = [a for a, _ in ins]
    for k, (a, t) in enumerate(ins):
        m = re.match(r"s_(?:cbranch_\w+|branch)\s+(-?\d+)", t)
        if not m:
            continue
        off = int(m.group(1))
        off = off - 65536 if off > 32767 else off  # (simm16 printed unsigned)
        tgt = a + 4 + 4 * off
        if tgt < a and a - tgt >= min_len:
            sub = [(x, y) for x, y in ins if tgt <= x <= a]
            v8, v8m = stats(sub + [(a + 4, "")])
            out.append((tgt, a, v8, v8m))
    return out
