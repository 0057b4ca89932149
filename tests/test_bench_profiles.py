"""CPU checks of the bench line's profile plumbing: the committed rocprofv3
kernel stats feed the ppo roofline's in-step kernel durations, and the PMC
traffic reduction keeps only the headline-sized dispatches (bench.py's
host-floor probe launches the same rollout kernel on 64 envs)."""
import csv
import json
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _traffic_update():
    spec = importlib.util.spec_from_file_location(
        "traffic_update", os.path.join(ROOT, "scripts", "traffic_update.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_committed_kernel_stats_cover_every_ppo_kernel():
    # round 4's summary: the unfused step; round 5's: the default step (the
    # first layer's backward inside the input-gradient GEMM, the operand
    # images built by the first layer's forward launch)
    # (round 6's record gather and 16x16x32 GEMMs postdate both)
    fused_away = {"split_x_kernel", "split_weights_kernel", "first_layer_bwd_kernel"}
    newer = {"gather_records_kernel", "gemm_x6_ws16_kernel", "gemm_x6_fl16_kernel",
             "gemm_x6_wgrad16_kernel"}
    r4 = bench.rocprof_averages(os.path.join(ROOT, "profiles", "r04_kernel_stats.csv"))
    for k in set(bench.PPO_KERNEL_NAMES.values()) - {"split_x_kernel", "gemm_x6_fl_kernel"} - newer:
        assert k in r4 and r4[k] > 0, k
    r5 = bench.rocprof_averages(os.path.join(ROOT, "profiles", "r05_kernel_stats.csv"))
    for k in set(bench.PPO_KERNEL_NAMES.values()) - fused_away - newer:
        assert k in r5 and r5[k] > 0, k
    # round 6's summary (the bench's default --kernel-stats): every kernel the
    # default step launches
    r6 = bench.rocprof_averages(os.path.join(ROOT, "profiles", "r06_kernel_stats.csv"))
    for k in set(bench.PPO_KERNEL_NAMES.values()) - fused_away:
        assert k in r6 and r6[k] > 0, k
    assert bench.rocprof_averages(os.path.join(ROOT, "profiles", "no_such.csv")) == {}


def test_round6_dominant_kernel_is_the_fused_input_gradient_gemm():
    """The committed round-6 summary picks the kernel with the largest time
    per optimizer step (the fused input-gradient GEMM, ~99 us) as the PPO
    block's dominant kernel."""
    class Cfg:
        batch_size, num_envs, n_steps, n_epochs = 65536, 65536, 32, 10
    rp = bench.rocprof_averages(os.path.join(ROOT, "profiles", "r06_kernel_stats.csv"))
    ks = {n: 1.0 for n in bench.PPO_KERNEL_NAMES}
    out = bench.ppo_roofline(Cfg, 0.13, ks, rp, {}, "profiles/r06_kernel_stats.csv")
    d = out["dominant_kernel"]
    assert d["kernel"] == "gemm_x6_fl16_kernel", d
    assert d["us"] == max(e["rocprof_us"] for e in out["kernels_per_minibatch"].values()
                          if "rocprof_us" in e and "bound" in e)


def test_ppo_roofline_carries_rocprof_durations_and_fractions():
    class Cfg:
        batch_size, num_envs, n_steps, n_epochs = 65536, 65536, 32, 10
    rp = {"gemm_x6_ws16_kernel": 80.0, "linear_tanh_kernel": 30.0}
    out = bench.ppo_roofline(Cfg, 0.15, {"gemm_x6_fwd": 100.0, "linear_tanh": 35.0,
                                         "grad_finish_clip_adam": 10.0}, rp,
                             {"gemm_x6_fwd": 90.0}, "profiles/x.csv")
    k = out["kernels_per_minibatch"]
    # 6 bf16 products x 2 nets x 2 M 256 256 FLOP over 80 us against 2.5 PF
    flop = 6 * 2 * 2 * 65536 * 256 * 256
    assert abs(k["gemm_x6_fwd"]["rocprof_frac"] - flop / 80e-6 / 2.5e15) < 1e-3
    assert k["gemm_x6_fwd"]["rocprof_us"] == 80.0 and k["gemm_x6_fwd"]["prefix_split_us"] == 100.0
    assert abs(k["gemm_x6_fwd"]["isolated_frac"] - flop / 90e-6 / 2.5e15) < 1e-3
    assert abs(k["linear_tanh"]["rocprof_frac"] - (15 * 4 + 2 * 256 * 4) * 65536 / 30e-6 / 8e12) < 1e-3
    assert "rocprof_us" not in k["grad_finish_clip_adam"]
    # no field called plain "frac" in the per-kernel entries: the prefix split
    # is labelled as such (verdict r04 item 6)
    assert all("frac" not in e for e in k.values())
    # the dominant kernel: the largest rocprof time per optimizer step
    d = out["dominant_kernel"]
    assert d["kernel"].startswith("gemm_x6_ws") and d["us"] == 80.0
    assert abs(d["frac"] - flop / 80e-6 / 2.5e15) < 1e-3 and d["isolated_us"] == 90.0
    # the whole-update ratio is named for what it is
    assert "frac" not in out and "fp32_equiv_frac_of_f32_peak" in out
    assert out["rocprof_source"] == "profiles/x.csv"


def test_ppo_roofline_without_rocprof_picks_the_largest_prefix_split():
    class Cfg:
        batch_size, num_envs, n_steps, n_epochs = 65536, 65536, 32, 10
    out = bench.ppo_roofline(Cfg, 0.15, {"gemm_x6_fwd": 100.0, "ppo_head": 120.0,
                                         "grad_finish_clip_adam": 500.0})
    d = out["dominant_kernel"]
    # the finish has no roofline bound and does not compete
    assert d["step"] == "ppo_head" and d["bound"] == "hbm" and d["us"] == 120.0
    assert d["unit"] == "GB/s" and abs(d["frac"] - 4140 * 65536 / 120e-6 / 8e12) < 1e-3
    assert bench.ppo_roofline(Cfg, 0.15, {"grad_finish_clip_adam": 5.0}).get(
        "dominant_kernel") is None


def test_dominant_kernel_follows_the_stats_csv(tmp_path):
    """verdict r05 item 4: the selection follows the rocprofv3 summary it is
    given -- one where the fused input-gradient kernel is the slowest names
    it, one where the forward GEMM is the slowest names that one."""
    class Cfg:
        batch_size, num_envs, n_steps, n_epochs = 65536, 65536, 32, 10
    steps = {"gather_minibatch": 7.0, "linear_tanh": 37.0, "gemm_x6_fwd": 110.0,
             "ppo_head": 51.0, "gemm_x6_bwd_first": 100.0, "gemm_x6_wgrad": 86.0,
             "grad_finish_clip_adam": 15.0}

    def stats(path, fl_ns, fwd_ns):
        with open(path, "w", newline="") as f:
            w = csv.DictWriter(f, ["Name", "Calls", "TotalDurationNs", "AverageNs",
                                   "Percentage"])
            w.writeheader()
            for name, ns in ((bench.PPO_KERNEL_NAMES["gemm_x6_bwd_first"], fl_ns),
                             (bench.PPO_KERNEL_NAMES["gemm_x6_fwd"], fwd_ns),
                             ("ppo_head_kernel", 50000)):
                w.writerow({"Name": "dr::(anonymous namespace)::%s(float const*)" % name,
                            "Calls": 10, "TotalDurationNs": 10 * ns, "AverageNs": ns,
                            "Percentage": 1})
        return bench.rocprof_averages(str(path))
    rp = stats(tmp_path / "a.csv", 111140, 88000)
    d = bench.ppo_roofline(Cfg, 0.14, steps, rp, {}, "a")["dominant_kernel"]
    assert d["step"] == "gemm_x6_bwd_first" and d["kernel"] == "gemm_x6_fl16_kernel"
    assert abs(d["us"] - 111.14) < 0.01 and abs(d["frac"] - 0.394) < 0.002
    rp = stats(tmp_path / "b.csv", 90000, 120000)
    d = bench.ppo_roofline(Cfg, 0.14, steps, rp, {}, "b")["dominant_kernel"]
    assert d["step"] == "gemm_x6_fwd" and d["us"] == 120.0


def test_traffic_average_keeps_the_largest_grid(tmp_path):
    d = tmp_path / "k32_FETCH_SIZE"
    d.mkdir()
    with open(d / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, ["Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for g, v in ((196608, 100.0), (196608, 102.0), (768, 1.0), (768, 1.0), (768, 1.0)):
            w.writerow({"Kernel_Name": "void dr::env_rollout_ab_kernel<double, false>(...)",
                        "Grid_Size": g, "Counter_Name": "FETCH_SIZE", "Counter_Value": v})
        w.writerow({"Kernel_Name": "gemm_x6_ws_kernel", "Grid_Size": 999999,
                    "Counter_Name": "FETCH_SIZE", "Counter_Value": 5.0})
    mean, n = _traffic_update().avg(str(d), "FETCH_SIZE")
    assert n == 2 and mean == 101.0


def _grid_stats():
    spec = importlib.util.spec_from_file_location(
        "kernel_grid_stats", os.path.join(ROOT, "scripts", "kernel_grid_stats.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_grid_stats_split_the_probe_from_the_headline_launches(tmp_path):
    p = tmp_path / "run_kernel_trace.csv"
    name = "void dr::env_rollout_ab_kernel<double, false>(...)"
    with open(p, "w", newline="") as f:
        w = csv.DictWriter(f, ["Kernel_Name", "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z",
                               "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for g, us in ((196608, 42.0), (196608, 44.0), (196608, 43.0), (768, 4.0), (768, 4.5)):
            w.writerow({"Kernel_Name": name, "Grid_Size_X": g, "Grid_Size_Y": 1,
                        "Grid_Size_Z": 1, "Start_Timestamp": 1000,
                        "End_Timestamp": 1000 + int(us * 1000)})
    rows = _grid_stats().summarise(str(p), ("env_rollout_ab_kernel",))
    assert [(r["grid"], r["dispatches"]) for r in rows] == [(196608, 3), (768, 2)]
    assert rows[0]["mean_us"] == 43.0 and rows[0]["median_us"] == 43.0
    out = tmp_path / "g.json"
    out.write_text(json.dumps(rows))
    k = bench.rollout_rocprof_k32(str(out), 65536, "f64")
    assert k["dispatches"] == 3 and k["mean_us"] == 43.0
    assert abs(k["frac"] - 65536 * (32 * 81 + 224) / 43e-6 / 8e12) < 1e-3
    assert bench.rollout_rocprof_k32(str(out), 4096, "f64") is None
    assert bench.rollout_rocprof_k32(str(tmp_path / "none.json"), 65536, "f64") is None


def test_pmc_valu_active_read_from_the_committed_summary():
    p = os.path.join(ROOT, "profiles", "r06_pmc_rollout.json")
    d = json.load(open(p))
    v = bench.pmc_rollout_valu_active(p)
    assert v["actions_from_hbm"] == d["actions_from_hbm"]["valu_active_frac_of_wave_cycles"]
    assert bench.pmc_rollout_valu_active(os.path.join(ROOT, "profiles", "none.json")) == {}


def test_kernel_source_hash_follows_the_sources(tmp_path, monkeypatch):
    h = bench.kernel_source_hash()
    assert len(h) == 64 and h == bench.kernel_source_hash()
    # a copy of the source set with one byte changed hashes differently
    import shutil
    root = tmp_path / "r"
    shutil.copytree(os.path.join(ROOT, "drone_rl_amd", "csrc"), root / "drone_rl_amd" / "csrc",
                    ignore=shutil.ignore_patterns("build"))
    (root / "include").mkdir()
    shutil.copy(os.path.join(ROOT, "include", "dronerl.h"), root / "include" / "dronerl.h")
    monkeypatch.setattr(bench, "ROOT", str(root))
    assert bench.kernel_source_hash() == h
    with open(root / "drone_rl_amd" / "csrc" / "trig.h", "a") as f:
        f.write("\n")
    assert bench.kernel_source_hash() != h


def test_stale_profiles_go_to_committed_artefacts(tmp_path, monkeypatch):
    prof = tmp_path / "p.json"
    prof.write_text("{}")
    prov = tmp_path / "provenance.json"
    monkeypatch.setattr(bench, "PROVENANCE_JSON", str(prov))
    monkeypatch.setattr(bench, "ARTEFACTS", {})
    prov.write_text(json.dumps({"p.json": {"source_hash": "0" * 64}}))
    assert bench.committed_or_stale("k", str(prof), {"mean_us": 1.0}) is None
    assert bench.ARTEFACTS["k"]["stale"] and bench.ARTEFACTS["k"]["values"] == {"mean_us": 1.0}
    prov.write_text(json.dumps({"p.json": {"source_hash": bench.kernel_source_hash()}}))
    live = bench.committed_or_stale("k2", str(prof), 0.5)
    assert live["value"] == 0.5 and live["provenance"]["matches_tree"]
    assert "k2" not in bench.ARTEFACTS


def test_every_committed_provenance_entry_names_a_profile():
    d = json.load(open(bench.PROVENANCE_JSON))
    for name, rec in d.items():
        assert os.path.exists(os.path.join(ROOT, "profiles", name)), name
        assert len(rec["source_hash"]) == 64


def test_rollout_kernel_name_reads_the_knob_like_atoi(monkeypatch):
    for v, ws in (("0", False), ("1", True), ("", False), ("false", False), (" 2x", True),
                  ("-0", False)):
        monkeypatch.setenv("DRONERL_ROLLOUT_WS", v)
        name = bench.rollout_kernel_name(65536, 256, False)
        assert name == ("env_rollout_ab_kernel" if ws else "env_rollout_kernel"), v
    monkeypatch.delenv("DRONERL_ROLLOUT_WS")
    assert bench.rollout_kernel_name(65536, 256, False) == "env_rollout_ab_kernel"
    assert bench.rollout_kernel_name(1 << 22, 256, False) == "env_rollout_kernel"
