"""bench.py's multi-rank launcher on the CPU (no GPU is touched): the rank environment, exit-status
propagation, termination of the surviving ranks when one fails, and the refusal when fewer GPUs
are visible than --gpus asks for."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))

import bench  # noqa: E402


def _py(code):
    return [sys.executable, "-c", code]


def test_launch_ranks_all_succeed_with_rank_env(tmp_path):
    code = ("import os, pathlib; e = os.environ; "
            f"pathlib.Path(r'{tmp_path}', 'r' + e['RANK']).write_text("
            "e['LOCAL_RANK'] + ' ' + e['WORLD_SIZE'] + ' ' + e['MASTER_ADDR'] + ' ' + e['MASTER_PORT'])")
    assert bench.launch_ranks(3, argv=_py(code), have=3, poll_s=0.05) == 0
    seen = [(tmp_path / f"r{r}").read_text().split() for r in range(3)]
    assert [s[0] for s in seen] == ["0", "1", "2"]
    assert all(s[1] == "3" and s[2] == "127.0.0.1" for s in seen)
    assert len({s[3] for s in seen}) == 1  # one rendezvous port for all ranks


def test_launch_ranks_propagates_failure_and_stops_the_others(tmp_path):
    # rank 1 fails at once with status 3; rank 0 would run 60 s unless terminated
    code = ("import os, sys, time, pathlib; r = int(os.environ['RANK']); "
            f"pathlib.Path(r'{tmp_path}', 'start' + str(r)).write_text('x'); "
            "sys.exit(3) if r == 1 else time.sleep(60)")
    t0 = time.time()
    assert bench.launch_ranks(2, argv=_py(code), have=2, poll_s=0.05) == 3
    assert time.time() - t0 < 30
    assert (tmp_path / "start1").exists()


def test_launch_ranks_refuses_too_few_gpus():
    assert bench.launch_ranks(4, argv=_py("raise SystemExit(0)"), have=1) == 2


def test_visible_gpus_does_not_initialise_hip():
    import torch
    n = bench.visible_gpus()
    assert n >= 0 and not torch.cuda.is_initialized()


class _FakeOps:
    """ops.ktime_read stand-in: per tag, (start_ms, stop_ms) relative to the first launch."""
    rec = {0: [(0.0, 0.3)], 1: [(1.0, 1.5), (1.2, 1.6)], 2: [(1.5, 2.1), (1.6, 2.4)]}

    def ktime_read(self, tag):
        return self.rec.get(tag, [])


def test_intervals_file_reproduces_the_roofline_union(tmp_path):
    """bench.py --intervals-out writes the timed region's attention intervals; tools/kunion.py
    recomputes the union per launch from that file alone (the line's roofline time), and --json
    carries flop / frac."""
    import json
    import subprocess
    path = tmp_path / "iv.csv"
    bench.write_intervals(_FakeOps(), str(path))
    # union of the bwd pair: [1.0, 2.4] = 1.4 ms over 2 launches = 700 us per launch
    iv = _FakeOps.rec[1] + _FakeOps.rec[2]
    assert abs(sum(b - a for a, b in [(1.0, 2.4)]) - 1.4) < 1e-12 and len(iv) == 4
    out = tmp_path / "u.json"
    subprocess.run([sys.executable, os.path.join(HERE, "..", "tools", "kunion.py"), str(path), "attn_bwd_dq_v4",
                    "attn_bwd_dkv_v4", "--flops", "7e8", "--json", str(out)], check=True, capture_output=True)
    d = json.loads(out.read_text())
    assert d["source_kind"] == "bench_intervals" and d["launches"] == 2
    assert abs(d["union_us_per_launch"] - 700.0) < 1e-6
    assert abs(d["tflops"] - 1.0) < 1e-6  # 7e8 flop / 700 us


def test_rocprof_union_reads_newest_trace_summary(tmp_path, monkeypatch):
    """The newest rocprofv3 union whose matched kernels are exactly the entry's current kernels;
    a newer file of other (replaced) kernels, one without the names, and bench-interval files are skipped."""
    import json
    prof = tmp_path / "profiles"
    prof.mkdir()
    cur = ["(anonymous namespace)::attn_bwd_dq_v4_kernel<4>(bf16 const*)",
           "(anonymous namespace)::attn_bwd_dkv_v4_kernel<4>(bf16 const*)"]
    old = ["(anonymous namespace)::attn_bwd_dq_v3_kernel<4>(bf16 const*)",
           "(anonymous namespace)::attn_bwd_dkv_v4_kernel<4>(bf16 const*)"]
    (prof / "r05_a_attn_bwd_union.json").write_text(json.dumps({"source_kind": "rocprofv3", "kernel_names": cur,
                                                                "union_us_per_launch": 900.0}))
    (prof / "r05_b_attn_bwd_union.json").write_text(json.dumps({"source_kind": "rocprofv3", "kernel_names": cur,
                                                                "union_us_per_launch": 850.0,
                                                                "generated_utc": "2026-10-18T00:00:00Z"}))
    (prof / "r05_c_attn_bwd_union.json").write_text(json.dumps({"source_kind": "bench_intervals", "kernel_names": cur,
                                                                "union_us_per_launch": 700.0}))
    (prof / "r05_d_attn_bwd_union.json").write_text(json.dumps({"source_kind": "rocprofv3", "kernel_names": old,
                                                                "union_us_per_launch": 600.0}))
    (prof / "r05_e_attn_bwd_union.json").write_text(json.dumps({"source_kind": "rocprofv3",
                                                                "union_us_per_launch": 500.0}))
    monkeypatch.setattr(bench, "HERE", str(tmp_path))
    us, src, gen = bench.rocprof_union("attn_bwd")
    assert us == 850.0 and src.endswith("r05_b_attn_bwd_union.json") and gen == "2026-10-18T00:00:00Z"
