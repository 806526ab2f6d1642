"""bench.py's multi-rank control flow on CPU (gloo): `python bench.py --gpus N`
without torchrun starts N ranks itself, every rank runs the same timed loop,
the max over ranks is reported and the JSON line carries the world size the
process group saw.  The HIP step is replaced by a CPU stub
(SFM_BENCH_CPU_STUB=1) -- only the launch / rank / timing path is exercised."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None, timeout=180):
    env = dict(os.environ, SFM_BENCH_CPU_STUB="1", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def _json_line(stdout):
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_spawns_two_ranks_without_torchrun():
    r = _run(["--gpus", "2", "--steps", "3", "--warmup", "1", "--config", "c3"])
    assert r.returncode == 0, r.stderr
    out = _json_line(r.stdout)
    assert out["n_gpus"] == 2
    assert out["dist"]["world_size"] == 2 and out["dist"]["backend"] == "gloo"
    assert out["dist"]["devices"] == ["cpu", "cpu"]
    assert out["config"]["pairs_per_gpu"] == 4 and out["config"]["global_batch"] == 8
    # every rank's pairs reach rank 0, in rank order
    assert out["gathered"]["pairs"] == 8
    assert out["gathered"]["rows"] == [[float(r), float(r), float(i)] for r in range(2) for i in range(4)]


def test_eight_rank_c3_shape():
    """The driver's SCALE run at its real shape (BASELINE C3: 8
    ranks x 4 bf16 pairs, embarrassingly data-parallel): 32 pairs gathered to
    rank 0 in rank order, every rank driving the device of its LOCAL_RANK."""
    r = _run(["--gpus", "8", "--steps", "2", "--warmup", "1", "--config", "c3"], timeout=300)
    assert r.returncode == 0, r.stderr
    out = _json_line(r.stdout)
    assert out["n_gpus"] == 8 and out["dist"]["world_size"] == 8
    assert out["config"]["pairs_per_gpu"] == 4 and out["config"]["global_batch"] == 32
    assert out["gathered"]["pairs"] == 32
    assert out["gathered"]["rows"] == [[float(r), float(r), float(i)] for r in range(8) for i in range(4)]


def test_single_rank_default():
    r = _run(["--steps", "2", "--warmup", "0"])
    assert r.returncode == 0, r.stderr
    out = _json_line(r.stdout)
    assert out["n_gpus"] == 1 and out["dist"]["world_size"] == 1
    assert out["config"]["name"] == "c2" and out["config"]["pairs_per_gpu"] == 8


def test_gpus_and_world_size_mismatch_fails():
    r = _run(["--gpus", "2", "--steps", "1"], extra_env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_pmc_summaries_sort_numerically():
    sys.path.insert(0, ROOT)
    import bench
    fs = ["profiles/r01_pmc_v6.json", "profiles/r01_pmc_v10.json", "profiles/r02_pmc.json", "profiles/r01_pmc.json"]
    assert sorted(fs, key=bench._round_version) == ["profiles/r01_pmc.json", "profiles/r01_pmc_v6.json",
                                                   "profiles/r01_pmc_v10.json", "profiles/r02_pmc.json"]
    # a config tag is part of the name, not the version
    assert bench._round_version("profiles/r02_pmc_c3_v1.json") == (2, 1)
    assert bench._round_version("profiles/r01_conv_pmc.json") == (-1, -1)


def test_pmc_traffic_matches_the_workload(tmp_path, monkeypatch):
    """The bench line's `traffic` comes only from a PMC summary collected on the
    same workload from the same sources (src_hash): c2 and c3 each
    find their own file, a config without one reports none, and a newer
    summary recorded from other sources is ignored."""
    import types
    sys.path.insert(0, ROOT)
    import bench

    def args(cfg, batch=None):
        b, _, it, nl, cd, _ = bench.CONFIGS[cfg]
        return types.SimpleNamespace(config=cfg, batch=batch or b, nlabel=nl, iters=it, cost_dtype=cd)

    prof = tmp_path / "profiles"
    prof.mkdir()

    def summary(name, cfg, h):
        b, _, it, nl, cd, _ = bench.CONFIGS[cfg]
        d = {"workload": {"config": cfg, "batch": b, "nlabel": nl, "iters": it, "cost_dtype": cd},
             "kernels": {"ransac_score": {"hbm_bytes": 1}}}
        if h:
            d["src_hash"] = h
        (prof / name).write_text(json.dumps(d))
    summary("r04_pmc_v1.json", "c2", "cur")
    summary("r04_pmc_v2.json", "c2", "old")      # newer, other sources
    summary("r04_pmc_v3.json", "c2", None)       # no hash: historical
    summary("r04_pmc_c3_v1.json", "c3", "cur")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "src_hash", lambda: "cur")
    _, src2 = bench.pmc_traffic(args("c2"))
    _, src3 = bench.pmc_traffic(args("c3"))
    assert src2 == os.path.join("profiles", "r04_pmc_v1.json")
    assert src3 == os.path.join("profiles", "r04_pmc_c3_v1.json")
    assert bench.pmc_traffic(args("c4")) == ({}, None)
    # same config, a batch no summary was collected on
    assert bench.pmc_traffic(args("c2", batch=3)) == ({}, None)


def test_src_hash_ignores_comments():
    sys.path.insert(0, ROOT)
    import bench
    h = bench.src_hash()
    assert len(h) == 16 and h == bench.src_hash()


def test_kernel_stats_files_sort_numerically():
    sys.path.insert(0, ROOT)
    import bench
    assert bench._stats_version("profiles/r03_kernel_stats_v10.csv") == ("c2", (3, 10))
    assert bench._stats_version("profiles/r03_kernel_stats_v9.csv") < bench._stats_version("profiles/r03_kernel_stats_v10.csv")
    assert bench._stats_version("profiles/r02_kernel_stats_sparse_v3.csv") == ("sparse", (2, 3))
    assert bench._stats_version("profiles/r01_regularize_kernel_stats.csv") is None


def test_rocprof_kernel_match_is_whole_name(tmp_path, monkeypatch):
    """k_score_mf must not match k_score_mf2's row (or the reverse): the
    rocprof frac is only reported from a summary holding every named kernel."""
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "r09_kernel_stats_v1.csv").write_text(
        '"Name","Calls","TotalDurationNs","AverageNs"\n'
        '"_ZN3sfm11k_score_mf2INS_9PackedSrcEEEvT_",2,10000000,5000000\n'
        '"_ZN3sfm10k_mf_candsEiPKi",2,20000,10000\n')
    (prof / "r09_kernel_stats_v1.meta.json").write_text(json.dumps({"src_hash": "cur"}))
    (prof / "r09_kernel_stats_v2.csv").write_text((prof / "r09_kernel_stats_v1.csv").read_text())
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "src_hash", lambda: "cur")

    class A:
        config = "c2"
    # v2 has no .meta.json (recorded from unknown sources): only v1 counts
    ms, src = bench.rocprof_kernel_ms(A, ("k_mf_cands", "k_score_mf2"))
    assert abs(ms - 5.01) < 1e-9 and src.endswith("r09_kernel_stats_v1.csv")
    assert bench.rocprof_kernel_ms(A, ("k_mf_cands", "k_score_mf"))[0] is None
    # the pruned scorer: k_score_mf2 launches, k_mf2_split, k_mf2_lead and k_mf2_keep per step
    (prof / "r09_kernel_stats_v3.csv").write_text(
        '"Name","Calls","TotalDurationNs","AverageNs"\n'
        '"_ZN3sfm11k_score_mf2INS_9PackedSrcEEEvT_",4,10000000,2500000\n'
        '"_ZN3sfm10k_mf2_leadINS_9PackedSrcEEEvT_",2,30000,15000\n'
        '"_ZN3sfm10k_mf2_keepENS_10PairParamsEii",2,10000,5000\n'
        '"_ZN3sfm11k_mf2_splitENS_10PairParamsEii",2,8000,4000\n'
        '"_ZN3sfm10k_mf_candsEiPKi",2,20000,10000\n')
    (prof / "r09_kernel_stats_v3.meta.json").write_text(json.dumps({"src_hash": "cur"}))
    ms, src = bench.rocprof_kernel_ms(A, ("k_mf_cands", "k_score_mf2"), optional=("k_mf2_split", "k_mf2_lead", "k_mf2_keep"))
    assert abs(ms - 5.034) < 1e-9 and src.endswith("r09_kernel_stats_v3.csv")
    monkeypatch.setattr(bench, "src_hash", lambda: "new")
    assert bench.rocprof_kernel_ms(A, ("k_mf_cands", "k_score_mf2")) == (None, None)


def test_valu_issue_from_pmc(tmp_path, monkeypatch):
    """The scorer's VALU-issue utilisation comes from the same matching PMC
    summary as `traffic`: SQ_INSTS_VALU x 4 cycles over the SIMDs' cycles
    (GRBM_GUI_ACTIVE summed over 8 XCDs); absent counters give None."""
    sys.path.insert(0, ROOT)
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "r09_pmc_v1.json").write_text(json.dumps(
        {"kernels": {"ransac_score": {"SQ_INSTS_VALU": 1024 * 1000, "GRBM_GUI_ACTIVE": 8 * 5000}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    v = bench.valu_issue(bench.pmc_kernel_counters(os.path.join("profiles", "r09_pmc_v1.json"), "ransac_score"))
    assert v["frac"] == 0.8 and v["simd_cycles_per_launch"] == 5000
    assert bench.valu_issue(bench.pmc_kernel_counters(None, "ransac_score")) is None
    assert bench.valu_issue({"SQ_INSTS_VALU": 5}) is None


def test_rank_device_index_and_shared_gpu(monkeypatch):
    """Each rank drives the device of its LOCAL_RANK; the shared-GPU rehearsal
    (SFM_BENCH_SHARED_GPU=1) puts every rank on device 0."""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.delenv("SFM_BENCH_SHARED_GPU", raising=False)
    assert [bench.rank_device_index(r) for r in range(8)] == list(range(8))
    monkeypatch.setenv("SFM_BENCH_SHARED_GPU", "1")
    assert [bench.rank_device_index(r) for r in range(4)] == [0, 0, 0, 0]


def test_tune_option_parses():
    sys.path.insert(0, ROOT)
    import bench
    a = bench.parse(["--tune", "sweep_store_px=2,sweep_nj=2", "--config", "c3"])
    assert a.tune == "sweep_store_px=2,sweep_nj=2" and a.config == "c3"
    assert bench.parse([]).tune == ""


def test_pipeline_and_overlap_ref_are_exclusive():
    """step_pipelined writes the whole volume and ignores overlap_ref, so the
    combination is refused rather than reported with the warped-half bytes."""
    import bench
    with pytest.raises(SystemExit):
        bench.parse(["--pipeline", "--overlap-ref", "score"])
    assert bench.parse(["--overlap-ref", "score"]).overlap_ref == "score"


def test_pmc_summary_sums_template_instances(tmp_path):
    """scripts/pmc_summary.py: a path key's per-step figure sums every
    dispatch of its kernels per step, and launches of template instances of
    one kernel (k_score_mf2<Src, false> and <Src, true>) add up in
    launches_sampled (round 5: the pruned scorer's three launches)."""
    import csv
    import importlib.util
    spec = importlib.util.spec_from_file_location("pmc_summary", os.path.join(ROOT, "scripts", "pmc_summary.py"))
    ps = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ps)
    src = tmp_path / "pmc"
    (src / "p1").mkdir(parents=True)
    a = "_ZN3sfm11k_score_mf2INS_9PackedSrcELb0EEEvT_NS_10PairParamsE"
    c = "_ZN3sfm11k_score_mf2INS_9PackedSrcELb1EEEvT_NS_10PairParamsE"
    m = "_ZN3sfm10k_mf_candsEiPKiPKdPDF16_NS_8MfParamsEPyPi"
    rows = []
    for step in range(2):                          # per step: cands, A, B (false), C (true)
        base = 10 * step
        rows += [(m, base + 1, 10.0), (a, base + 2, 100.0), (a, base + 3, 1.0), (c, base + 4, 5.0)]
    with open(src / "p1" / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Dispatch_Id", "Counter_Name", "Counter_Value"])
        for name, d, v in rows:
            w.writerow([name, d, "SQ_WAVES", v])
    dst = tmp_path / "out.json"
    ps.main(str(src), str(dst), "c2")
    k = json.load(open(dst))["kernels"]["ransac_score"]
    assert k["launches_sampled"] == {"k_mf_cands": 2, "k_score_mf2": 6}
    assert abs(k["SQ_WAVES"] - 116.0) < 1e-9               # 10 + 100 + 1 + 5 per step


def test_one_sided_pruning_work_accounting():
    """The scorer's roofline line under the one-sided pruning (round 6): the
    algorithmic work stays (candidates x N - skipped) x 50 FLOP, the MFMA pipe
    use counts 96 FLOP per one-sided and 128 per two-sided evaluation, and the
    work string names both passes."""
    sys.path.insert(0, ROOT)
    import bench
    done, evals, skipped = 3000, 3200, 200
    r0 = bench.score_roofline(True, 1.0, done, evals, skipped, 10, 320, 2.0, None, None, scorer="k_score_mf2+prune")
    r1 = bench.score_roofline(True, 1.0, done, evals, skipped, 10, 320, 2.0, None, None, scorer="k_score_mf2+prune",
                              upper=(done, 2 * 320, 2))
    assert r0["mfma_issued"]["tflops"] == round(done * 128 / 2e-3 / 1e12, 1)
    assert r1["mfma_issued"]["tflops"] == round((done * 96 + 2 * 320 * 128) / 2e-3 / 1e12, 1)
    assert "one-sided pass" in r1["work"] and "2 of 10 candidates kept" in r1["work"]
    assert "one-sided" in r1["kernel"] and "one-sided" not in r0["kernel"]


def test_clock_probe_edits_apply_to_the_sources():
    """scripts/build_clock_probe.py patches a temporary copy of score_mf2.h at
    fixed anchors: each must still occur exactly once in the current source,
    or the diagnostic behind profiles/r06_scorer_clock.txt no longer builds."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("build_clock_probe",
                                                  os.path.join(ROOT, "scripts", "build_clock_probe.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    src = open(os.path.join(ROOT, "deep-sfm-revisited_amd", "csrc", "score_mf2.h")).read()
    for old, _ in mod.EDITS:
        assert src.count(old) == 1, old
