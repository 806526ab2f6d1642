"""Copy one scripts/gpu_evidence.sh session's results from gpurun_out/ into
profiles/ (the tracked, judged copies), each under the next free version:

  profiles/<R>_bench_<cfg>_vK.json        the bench JSON lines
  profiles/<R>_kernel_stats[_<cfg>]_vK.csv  rocprofv3 --stats summaries, with a
      .meta.json sidecar holding the src_hash of the profiled bench line (the
      sources the profile was recorded from; bench.py only uses a summary
      whose hash matches its own sources)
  profiles/<R>_pmc[_<cfg>]_vK.json       PMC summaries (scripts/pmc_summary.py)
  profiles/<R>_gpu_tests_vK.txt          the pytest -m gpu tail

Usage: python scripts/collect_evidence.py r04"""
import glob
import json
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def next_path(stem, ext):
    k = 1
    while os.path.exists(os.path.join(PROF, f"{stem}_v{k}{ext}")):
        k += 1
    return os.path.join(PROF, f"{stem}_v{k}{ext}")


def json_line(log):
    lines = [l for l in open(log) if l.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def main(R):
    done = []
    for cfg in ("c2", "sparse", "c3", "c4", "c5"):
        log = os.path.join(OUT, f"{R}_bench_{cfg}.log")
        if os.path.exists(log) and json_line(log):
            p = next_path(f"{R}_bench_{cfg}", ".json")
            json.dump(json_line(log), open(p, "w"))
            done.append(p)
        stats = glob.glob(os.path.join(OUT, f"{R}_prof_{cfg}", "**", "*kernel_stats*.csv"), recursive=True)
        plog = os.path.join(OUT, f"{R}_prof_{cfg}.log")
        if stats and os.path.exists(plog):
            line = json_line(plog)
            p = next_path(f"{R}_kernel_stats" + ("" if cfg == "c2" else f"_{cfg}"), ".csv")
            shutil.copy(stats[0], p)
            json.dump({"src_hash": line.get("src_hash") if line else None, "bench_line": line}, open(p[:-4] + ".meta.json", "w"))
            done.append(p)
        pmc = os.path.join(OUT, f"{R}_pmc_{cfg}")
        if os.path.isdir(pmc):
            p = next_path(f"{R}_pmc" + ("" if cfg == "c2" else f"_{cfg}"), ".json")
            subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_summary.py"), pmc, p, cfg], check=True)
            done.append(p)
    t = os.path.join(OUT, f"{R}_pytest_gpu.log")
    if os.path.exists(t):
        p = next_path(f"{R}_gpu_tests", ".txt")
        lines = open(t).read().splitlines()
        open(p, "w").write("\n".join(lines[-40:]) + "\n")
        done.append(p)
    for p in done:
        print(os.path.relpath(p, ROOT))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r05")
