"""Round-5 finding (the 4-byte pair-staging miscompute of round 4): on gfx950
a VMEM store of more than 64 bits of data (buffer/global_store_dwordx3/x4)
followed IMMEDIATELY by a VALU instruction that overwrites one of its data
VGPRs stored the overwritten value for part of the wave -- with an SGPR
soffset, the case LLVM's hazard recognizer treats as hazard-free (it inserts
the wait state only without an SGPR soffset).  This lists every such
instruction pair in a hipcc -S (gfx950) assembly file, per kernel.
usage: store_hazard_check.py file.s|lib.so [...]"""
import re
import sys

STORE = re.compile(r"^(buffer|global|flat|scratch)_store_(dwordx3|dwordx4|b96|b128)\s+(.*)$")


def vregs(tok):
    """The vector registers an operand names, as (file, index) pairs: VGPRs
    ('v', i) from v[i:j] / vN and AGPRs ('a', i) from a[i:j] / aN (a store
    can take its data from AGPRs, and v_accvgpr_write / v_mfma write them)."""
    m = re.match(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"([va])(\d+)$", tok)
    return {(m.group(1), int(m.group(2)))} if m else set()


def check(path, lines=None):
    """(kernel, store, next instruction) triples of a hipcc -S file or of
    llvm-objdump -d output (``lines``)."""
    hits = []
    kernel = None
    prev = None
    for raw in (lines if lines is not None else open(path)):
        line = raw.split(";")[0].split("//")[0].strip()
        m = re.match(r"^(?:[0-9a-f]+ )?<?(_Z[^>:\s]+)>?:", line)
        if m:
            kernel, prev = m.group(1), None
            continue
        if not line or line.startswith(".") or line.endswith(":"):
            continue
        if prev is not None:
            op = line.split()[0]
            if op.startswith("v_"):
                dst = line.split()[1].rstrip(",")
                if vregs(dst) & prev[1]:
                    hits.append((kernel, prev[0], line))
        s = STORE.match(line)
        if s:
            ops = [t.strip() for t in s.group(3).split(",")]
            data = ops[1] if s.group(1) == "global" or s.group(1) == "flat" else ops[0]
            prev = (line, vregs(data))
        else:
            prev = None
    return hits


def library_device_code(so_path):
    """llvm-objdump -d lines of every gfx950 code object bundled in a HIP
    shared library (.hip_fatbin section, one offload bundle per translation
    unit)."""
    import os
    import subprocess
    import tempfile
    llvm = "/opt/rocm/lib/llvm/bin"
    out = []
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fatbin")
        subprocess.run([f"{llvm}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", so_path, os.path.join(d, "x")],
                       check=True, capture_output=True)
        data = open(fb, "rb").read()
        offs = [m.start() for m in re.finditer(re.escape(b"__CLANG_OFFLOAD_BUNDLE__"), data)]
        for i, o in enumerate(offs):
            b = os.path.join(d, f"b{i}")
            co = os.path.join(d, f"c{i}.co")
            open(b, "wb").write(data[o:offs[i + 1] if i + 1 < len(offs) else len(data)])
            subprocess.run([f"{llvm}/clang-offload-bundler", "--unbundle", "--type=o",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={b}", f"--output={co}"],
                           check=True, capture_output=True)
            dis = subprocess.run([f"{llvm}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True,
                                 capture_output=True, text=True).stdout
            out.extend(dis.split("\n"))
    return out


if __name__ == "__main__":
    total = 0
    for p in sys.argv[1:]:
        for k, st, nxt in check(p, library_device_code(p) if p.endswith(".so") else None):
            total += 1
            print(f"{p}: {k[:70]}\n    {st}\n    {nxt}")
    print(f"{total} store-data overwrite(s) with no wait state")
    sys.exit(1 if total else 0)
