"""The measurement tools behind the committed profiles (CPU only, synthetic rocprofv3 CSVs):
tools/pmc_summary.py (FETCH_SIZE / WRITE_SIZE per kernel with the gfx950 corrections and the
per-launch large / small split used for the LiDAR / map patch weight gradient) and tools/kunion.py
(union of kernel execution intervals, the bench's roofline time)."""
import csv
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
TOOLS = os.path.join(HERE, "..", "tools")


def _write_counters(path, counter, rows):
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "run_counter_collection.csv"), "w", newline="") as fh:
        w = csv.DictWriter(fh, ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value", "Start_Timestamp",
                                "End_Timestamp"])
        w.writeheader()
        for did, name, val, s, e in rows:
            w.writerow(dict(Dispatch_Id=did, Kernel_Name=name, Counter_Name=counter, Counter_Value=val,
                            Start_Timestamp=s, End_Timestamp=e))


def test_pmc_summary_corrections_and_per_launch_split(tmp_path):
    k = "void ivit::patch_wgrad_kernel<3, 2, 0>(float const*)"
    a = "attn_fwd_kernel(int)"
    # dispatch order: map (small) then LiDAR (large), twice; written out of order on purpose
    fetch = [(4, k, 3.0e6, 0, 900_000), (1, k, 100.0e3, 0, 40_000), (2, k, 3.2e6, 0, 1_000_000),
             (3, k, 110.0e3, 0, 46_000), (5, a, 1000.0, 0, 10)]
    write = [(1, k, 20.0e3, 0, 1), (2, k, 70.0e3, 0, 1), (3, k, 30.0e3, 0, 1), (4, k, 80.0e3, 0, 1),
             (5, a, 500.0, 0, 1)]
    _write_counters(str(tmp_path / "f"), "FETCH_SIZE", fetch)
    _write_counters(str(tmp_path / "w"), "WRITE_SIZE", write)
    out = subprocess.run([sys.executable, os.path.join(TOOLS, "pmc_summary.py"), str(tmp_path / "f"),
                          str(tmp_path / "w"), "patch_wgrad"], capture_output=True, text=True, check=True).stdout
    d = json.loads(out)["kernels"]
    pk = d["ivit::patch_wgrad_kernel<3, 2, 0>"]
    # read = 2 x FETCH_SIZE KiB (gfx950 wide-load correction), write = WRITE_SIZE KiB
    assert pk["launches"] == 4
    assert abs(pk["hbm_read_bytes_avg"] - 2 * 1024 * (3.0e6 + 100e3 + 3.2e6 + 110e3) / 4) < 1
    assert abs(pk["hbm_write_bytes_avg"] - 1024 * 50e3) < 1
    pl = pk["per_launch"]
    assert [r["launch"] for r in pl["launches"]] == [0, 1, 2, 3]
    assert [round(r["read_bytes"] / 2048) for r in pl["launches"]] == [100_000, 3_200_000, 110_000, 3_000_000]
    assert pl["large"]["launches"] == 2 and pl["small"]["launches"] == 2
    assert abs(pl["large"]["read_bytes_avg"] - 2 * 1024 * 3.1e6) < 1
    assert abs(pl["large"]["write_bytes_avg"] - 1024 * 75e3) < 1
    assert abs(pl["small"]["dur_us_avg"] - 43.0) < 1e-6
    assert "per_launch" not in d["attn_fwd_kernel"]


def test_kunion_counts_overlap_once(tmp_path):
    p = tmp_path / "run_kernel_trace.csv"
    with open(p, "w", newline="") as fh:
        w = csv.DictWriter(fh, ["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        # two launches of the (dq, dkv) pair on two streams; the second pair overlaps the first
        for name, s, e in [("attn_bwd_dq_v3", 0, 100), ("attn_bwd_dkv_v3", 100, 250),
                           ("attn_bwd_dq_v3", 200, 300), ("attn_bwd_dkv_v3", 300, 400),
                           ("other_kernel", 0, 1000)]:
            w.writerow(dict(Kernel_Name=name, Start_Timestamp=s * 1000, End_Timestamp=e * 1000))
    out = subprocess.run([sys.executable, os.path.join(TOOLS, "kunion.py"), str(p), "attn_bwd_dq_v3",
                          "attn_bwd_dkv_v3"], capture_output=True, text=True, check=True).stdout
    # union [0, 400] us over 2 launches = 200 us per launch; own intervals 100 + 150 + 100 + 100
    assert "2 launches" in out and "200.0 us per launch" in out and "225.0 us per launch" in out
