"""Extract one kernel's instruction stream from a hipcc -S (gfx950) assembly
file, comments and labels stripped, registers optionally normalised: used to
check that a source clean-up leaves a kernel's machine code unchanged.
usage: python scripts/isa_kernel.py file.s name_substring [--norm] [--stats]"""
import re
import sys


def kernel_lines(path, sub):
    lines = open(path).read().split("\n")
    out, inside = [], False
    for ln in lines:
        if not inside:
            m = re.match(r"^(_Z\S+):\s*(;.*)?$", ln)
            if m and sub in m.group(1) and not ln.startswith(".L"):
                inside = True
                out.append(m.group(1))
            continue
        if ln.startswith(".Lfunc_end"):
            break
        t = ln.split(";")[0].rstrip()
        if not t.strip() or (t.strip().startswith(".") and not t.strip().endswith(":")):
            continue
        out.append(t.strip())
    return out


def norm(l):
    return re.sub(r"\b([vsa])\[?\d+(:\d+)?\]?", r"\1R", l)


if __name__ == "__main__":
    path, sub = sys.argv[1], sys.argv[2]
    ls = kernel_lines(path, sub)
    if "--stats" in sys.argv:
        from collections import Counter
        c = Counter(l.split()[0] for l in ls[1:] if not l.endswith(":"))
        print(ls[0], sum(c.values()), "instructions")
        for k, v in sorted(c.items()):
            print(f"{v:6d} {k}")
    else:
        for l in ls:
            print(norm(l) if "--norm" in sys.argv else l)
