"""Per-kernel register, spill and scratch figures of the gfx950 code objects
in a HIP shared library (code-object metadata notes), e.g.
    python scripts/kernel_resources.py deep-sfm-revisited_amd/sfm_amd/libsfm_hip.so score_mf2
Prints name, VGPRs, SGPRs, VGPR / SGPR spills, scratch bytes per lane, LDS bytes."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
KEYS = [".vgpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count", ".private_segment_fixed_size",
        ".group_segment_fixed_size"]


def resources(so_path, pattern=""):
    out = []
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fatbin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", so_path, os.path.join(d, "x")],
                       check=True, capture_output=True)
        data = open(fb, "rb").read()
        offs = [m.start() for m in re.finditer(re.escape(b"__CLANG_OFFLOAD_BUNDLE__"), data)]
        for i, o in enumerate(offs):
            b, co = os.path.join(d, f"b{i}"), os.path.join(d, f"c{i}.co")
            open(b, "wb").write(data[o:offs[i + 1] if i + 1 < len(offs) else len(data)])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={b}", f"--output={co}"],
                           check=True, capture_output=True)
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                                   text=True).stdout
            for blk in re.split(r"\n\s+- \.", notes)[1:]:
                blk = "." + blk
                m = re.search(r"\.name:\s+(\S+)", blk)
                if not m or pattern not in m.group(1) or m.group(1).endswith(".kd"):
                    continue
                vals = {}
                for k in KEYS:
                    v = re.search(re.escape(k) + r":\s+(\S+)", blk)
                    vals[k] = int(v.group(1)) if v else None
                out.append((m.group(1), vals))
    return out


if __name__ == "__main__":
    for name, v in resources(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""):
        print(f"{name[:90]:90s} vgpr {v['.vgpr_count']} sgpr {v['.sgpr_count']} spill v/s "
              f"{v['.vgpr_spill_count']}/{v['.sgpr_spill_count']} scratch {v['.private_segment_fixed_size']} "
              f"lds {v['.group_segment_fixed_size']}")
