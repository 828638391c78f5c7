"""bench.py's --gpus / WORLD_SIZE logic (no GPU): --gpus N is authoritative — without a launcher
and N > 1 the bench starts N ranks itself; a launcher's WORLD_SIZE must equal N; nccl needs one GPU
per rank."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_single_gpu_runs_in_process():
    assert bench.resolve_world(1, {}, "nccl", lambda: 0) == ("run", 1)


def test_no_launcher_spawns_n_ranks():
    assert bench.resolve_world(8, {}, "nccl", lambda: 8) == ("spawn", 8)
    assert bench.resolve_world(2, {}, "gloo", lambda: 1) == ("spawn", 2)  # ranks share a GPU


def test_under_launcher_world_must_match():
    assert bench.resolve_world(4, {"WORLD_SIZE": "4"}, "nccl", lambda: 8) == ("run", 4)
    with pytest.raises(SystemExit):
        bench.resolve_world(8, {"WORLD_SIZE": "1"}, "nccl", lambda: 8)
    with pytest.raises(SystemExit):
        bench.resolve_world(1, {"WORLD_SIZE": "2"}, "gloo", lambda: 1)


def test_nccl_needs_a_gpu_per_rank():
    with pytest.raises(SystemExit):
        bench.resolve_world(8, {}, "nccl", lambda: 1)
    with pytest.raises(SystemExit):
        bench.resolve_world(2, {"WORLD_SIZE": "2"}, "nccl", lambda: 1)
    with pytest.raises(SystemExit):
        bench.resolve_world(0, {}, "nccl", lambda: 1)
