"""The measurement plumbing on the CPU: bench.py attaches the committed PMC / SQ profiles to its
roofline block only for the library build and workload they measured, and
tools/summarize_profile.py picks the K timed integrate launches out of a kernel trace -- by the
index the bench line records, or (passes run without HIP events) as the process's last K launches
after the timed call's two pipeline-fill launches."""
import csv
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture()
def bench(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    sys.path.insert(0, REPO)
    import bench as b
    return b


def _roof():
    return {"bound": "hbm", "achieved": 3000.0, "peak": 8000.0, "frac": 0.375, "kernel_avg_us": 650.0,
            "bytes_per_launch": 1.95e9, "launches": 20}


def _profiles(tmp_path, build, workload):
    pmc = tmp_path / "pmc.json"
    sq = tmp_path / "sq.json"
    pmc.write_text(json.dumps({"build_id": build, "workload": workload, "l2_memside_bytes_per_launch": 2.2e9,
                               "raw_bytes_per_launch": 1.3e9}))
    sq.write_text(json.dumps({"build_id": build, "workload": workload, "valu_busy_per_simd": 0.88,
                              "median_per_launch": {"SQ_INSTS_VALU": 3.4e8}}))
    return str(pmc), str(sq)


def test_profiles_attach_only_for_the_same_build_and_workload(bench, tmp_path, monkeypatch):
    st = {"voxel_updates": 20 * 16 * 15_000_000, "kernel_launches": 20}
    pmc, sq = _profiles(tmp_path, "abc", bench.WORKLOAD)
    roof = _roof()
    bench.attach_profiles(roof, st, "abc", pmc, sq, bench.WORKLOAD)
    assert roof["traffic"] == 2_200_000_000 and roof["bound"] == "valu" and roof["traffic_raw"] == 1_300_000_000
    assert roof["traffic_over_algorithmic"] == pytest.approx(2.2e9 / 1.95e9, abs=1e-3)
    assert roof["traffic_frac"] == pytest.approx(2.2e9 / 650e-6 / 8e12, abs=1e-4)
    assert roof["valu"]["valu_busy"] == 0.88 and "profiles_note" not in roof
    roof = _roof()
    bench.attach_profiles(roof, st, "other", pmc, sq, bench.WORKLOAD)  # another build: nothing attached, and said why
    assert "traffic" not in roof and "valu" not in roof and roof["bound"] == "hbm"
    assert "measured library build abc, this is other" in roof["profiles_note"]
    pmc, sq = _profiles(tmp_path, "abc", "another workload")
    roof = _roof()
    bench.attach_profiles(roof, st, "abc", pmc, sq, bench.WORKLOAD)
    assert "traffic" not in roof and "measured another workload" in roof["profiles_note"]


def test_roofline_prices_each_batched_voxel_once(bench):
    """temporal batching must never push roofline.achieved past peak.  A launch of 16
    frames whose batch updates U distinct voxels moves 24 B of state per distinct voxel, however
    many of its frames update each one: the frac follows U, and the per-frame pricing (24 B per
    update) is only a named secondary figure."""
    L, F = 20, 320
    st = {"voxel_updates": F * 15_700_000, "batch_voxels": L * 80_000_000, "kernel_launches": L,
          "kernel_ms": L * 0.652}
    r = bench.integrate_roofline(st, F, "k")
    alg = 24.0 * L * 80_000_000 + 5.0 * bench.PIX * F
    assert r["bytes_per_launch"] == round(alg / L)
    assert r["frac"] == pytest.approx(alg / (L * 0.652e-3) / 8e12, abs=1e-4) and r["frac"] < 1
    assert r["per_frame_bytes_frac"] > 1 > r["frac"]  # what round 4's line reported as frac
    h = bench.integrate_roofline(st, F, "k", blocks_touched=1000)
    assert h["bytes_per_launch"] == round((alg + 16.0 * 1000) / L)
    assert bench.integrate_roofline(dict(st, kernel_launches=0), F, "k") is None


def test_bound_names_the_resource_closest_to_its_peak(bench, tmp_path):
    st = {"voxel_updates": 20 * 16 * 15_000_000, "kernel_launches": 20}
    pmc, sq = _profiles(tmp_path, "abc", bench.WORKLOAD)
    roof = dict(_roof(), frac=0.95)  # memory nearer its peak than the VALU's 0.88
    bench.attach_profiles(roof, st, "abc", pmc, sq, bench.WORKLOAD)
    assert roof["bound"] == "hbm" and "bound_note" not in roof


def _pmc_csv(path, values, kernel):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for d, v in enumerate(values):
            for half in (0.5, 0.5):  # (summed over dimensions)
                w.writerow({"Dispatch_Id": 100 + d, "Kernel_Name": "void " + kernel, "Counter_Name": "FETCH_SIZE",
                            "Counter_Value": v * half})
            w.writerow({"Dispatch_Id": 100 + d, "Kernel_Name": "tsdf::k_other", "Counter_Name": "FETCH_SIZE",
                        "Counter_Value": 1.0})


def test_summaries_pick_the_timed_launches(tmp_path):
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import summarize_profile as sp
    K = sp.K
    warm = [500.0] * 7
    timed = [1000.0 + i for i in range(K)]
    # a pass without HIP events: the timed call is last; its two fill launches come first
    p = str(tmp_path / "a.csv")
    _pmc_csv(p, warm + [5.0, 7.0] + timed, sp.KERNEL)
    assert sp.pmc_timed(p, "FETCH_SIZE", None) == timed
    # by the bench line's index (here 9: after 7 warm-up and 2 fill launches), whatever follows
    _pmc_csv(p, warm + [5.0, 7.0] + timed + [500.0] * 3, sp.KERNEL)
    assert sp.pmc_timed(p, "FETCH_SIZE", 9) == timed
    # the last K are not preceded by two fill launches: refused
    _pmc_csv(p, warm + [500.0, 500.0] + timed, sp.KERNEL)
    with pytest.raises(RuntimeError):
        sp.pmc_timed(p, "FETCH_SIZE", None)
    assert sp.first_index({"first_timed_launch_index": 4}) == 4
    assert sp.first_index({"roofline": {"first_timed_launch_index": 5}}) == 5
    assert sp.first_index({"roofline": None}) is None


def test_hash_profile_takes_the_inserting_window():
    """tools/summarize_profile.py hash: the bench's hash leg ends with the timed call (K + 2
    launches of k_fused_hash<0, true>: two pipeline fills, then K integrating) and the no-allocation
    repeat (K + 2 more); the inserting window is the first call's K integrating launches."""
    import tempfile
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import summarize_profile as sp
    K = sp.K
    vals = [9.0] * 5 + [1.0, 2.0] + [100.0 + i for i in range(K)] + [3.0, 4.0] + [200.0 + i for i in range(K)]
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "h.csv")
        with open(p, "w", newline="") as f:
            w = csv.DictWriter(f, ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
            w.writeheader()
            for i, v in enumerate(vals):
                w.writerow({"Dispatch_Id": 10 + i, "Kernel_Name": "void tsdf::k_fused_hash<0, true>(...)",
                            "Counter_Name": "FETCH_SIZE", "Counter_Value": v})
                w.writerow({"Dispatch_Id": 10 + i, "Kernel_Name": "void tsdf::k_fused<true, 4, 0, true>(...)",
                            "Counter_Name": "FETCH_SIZE", "Counter_Value": -1.0})
        ins, rep = sp.hash_windows(p)
    assert [r["FETCH_SIZE"] for r in ins] == [100.0 + i for i in range(K)]
    assert [r["FETCH_SIZE"] for r in rep] == [200.0 + i for i in range(K)]


def test_load_sweep_attached_only_for_its_build(bench, tmp_path):
    """config[2]'s load-factor sweep rides in the hash block only for the library build it measured."""
    pt = {"slots": 1 << 19, "target_load": 0.75, "load_window_end": 0.75,
          "inserting": {"kernel_avg_us": 1460.0, "over_dense": 1.10, "over_load_0_1": 1.0, "mean_probe": 2.7,
                        "max_probe": 95, "tombstones_after": 2190},
          "repeat": {"kernel_avg_us": 1418.0}}
    p = tmp_path / "sweep.json"
    p.write_text(json.dumps({"build_id": "abc", "workload": "w", "dense_same_extent": {"async": {"kernel_avg_us": 1325.0}},
                             "sweep": [pt]}))
    got = bench.load_sweep("abc", str(p))
    assert got["points"][0]["inserting_over_dense"] == 1.10 and got["dense_same_extent_kernel_us"] == 1325.0
    assert "measured library build abc, this is xyz" in bench.load_sweep("xyz", str(p))["note"]
    assert "no " in bench.load_sweep("abc", str(tmp_path / "none.json"))["note"]
