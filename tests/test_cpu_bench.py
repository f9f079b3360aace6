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
