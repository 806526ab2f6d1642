"""Build the diagnostic library that scripts/probe_scorer_clock.py reads:
a copy of csrc/ (in a temporary directory; the tree's sources, and so its
src_hash, stay untouched) whose one-sided non-mapped k_score_mf2 launch stamps
s_memtime / s_memrealtime once around its unit loop per block (the recipe of
MI355X_MICROARCH.md: in-kernel clock = d memtime / d memrealtime x 100 MHz)
and counts its waves' runs, exported as sfm_experiment_clk.
Output: abl/libsfm_hip_clk.so (git-ignored)."""
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

EDITS = [
    ("// The float64 test of queued",
     """__device__ unsigned long long g_clk[4096][3];   // per block: d memtime, d memrealtime, runs
extern "C" int sfm_experiment_clk(unsigned long long* out, int reset) {
  if (reset) {
    static unsigned long long z[4096][3];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_clk), z, sizeof(z)) == hipSuccess ? 0 : 2;
  }
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_clk), sizeof(g_clk)) == hipSuccess ? 0 : 2;
}

// The float64 test of queued"""),
    ("  if (s_first[batch] == 0) return;\n",
     """  if (s_first[batch] == 0) return;
  const unsigned long long clk_c0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  unsigned long long clk_runs = 0;
"""),
    ("        const int lane = mf2_lane(), hl = lane >> 5, rl = lane & 31;\n        // the next run's rows load",
     "        ++clk_runs;\n        const int lane = mf2_lane(), hl = lane >> 5, rl = lane & 31;\n"
     "        // the next run's rows load"),
    ("  // (the loop left right after a block barrier)\n  if (tb >= 0) flush(tb);",
     """  // (the loop left right after a block barrier)
  if constexpr (kUpper && !kMap) {
    const unsigned long long clk_c1 = __builtin_amdgcn_s_memtime(), clk_r1 = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if (blockIdx.x < 4096) {
      if (tid == 0) { g_clk[blockIdx.x][0] = clk_c1 - clk_c0; g_clk[blockIdx.x][1] = clk_r1 - clk_r0; }
      if ((tid & 63) == 0) atomicAdd(&g_clk[blockIdx.x][2], clk_runs);
    }
  }
  if (tb >= 0) flush(tb);"""),
]


def main():
    with tempfile.TemporaryDirectory() as tmp:
        pkg = os.path.join(tmp, "deep-sfm-revisited_amd")
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
        shutil.copytree(os.path.join(ROOT, "deep-sfm-revisited_amd", "csrc"), os.path.join(pkg, "csrc"),
                        ignore=shutil.ignore_patterns("build*"))
        p = os.path.join(pkg, "csrc", "score_mf2.h")
        s = open(p).read()
        for old, new in EDITS:
            assert s.count(old) == 1, old
            s = s.replace(old, new)
        open(p, "w").write(s)
        os.makedirs(os.path.join(ROOT, "abl"), exist_ok=True)
        out = os.path.join(ROOT, "abl", "libsfm_hip_clk.so")
        subprocess.run(["make", "-s", "-B", "-j8", "-C", os.path.join(pkg, "csrc"), "ARCH=gfx950", f"OUT={out}"],
                       check=True)
        print(out)


if __name__ == "__main__":
    main()
