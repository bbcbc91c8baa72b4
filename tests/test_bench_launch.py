"""bench.py starts its own N ranks when it is run as ``python bench.py --gpus N`` without a
launcher: torch.distributed.run as a child process (never an exec), one rank per GPU,
rendezvous on 127.0.0.1, the same arguments forwarded; with WORLD_SIZE set (the driver's
torch.distributed.run form) it runs as the rank it is."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (module level imports the standard library only)


def test_launch_decision():
    assert bench.needs_launch(8, {})
    assert bench.needs_launch(2, {"RANK": "0"})
    assert not bench.needs_launch(1, {})
    assert not bench.needs_launch(8, {"WORLD_SIZE": "8"})
    assert not bench.needs_launch(2, {"WORLD_SIZE": "1"})


def test_launch_command_forwards_arguments():
    argv = ["--gpus", "4", "--steps", "20", "--warmup", "3", "--group", "8"]
    cmd = bench.launch_command(4, argv, 29512, python="/usr/bin/python3")
    assert cmd[:3] == ["/usr/bin/python3", "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "4"
    assert cmd[cmd.index("--nnodes") + 1] == "1"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29512"
    script = os.path.join(ROOT, "bench.py")
    assert cmd[cmd.index(script) + 1:] == argv


def test_launch_runs_a_child_and_returns_its_code(monkeypatch):
    calls = []

    def fake_call(cmd, env=None):
        calls.append((cmd, env))
        return 3

    import subprocess
    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.setattr(os, "execv", lambda *a: pytest.fail("bench must not exec"))
    assert bench.launch_ranks(2, ["--gpus", "2"]) == 3
    (cmd, env), = calls
    assert "torch.distributed.run" in cmd and cmd[-2:] == ["--gpus", "2"]
    assert env is not None and "WORLD_SIZE" not in env


def test_main_launches_before_touching_torch(monkeypatch):
    # the launch happens before bench imports torch (nothing has touched the GPU)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "1"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    seen = {}

    def fake_launch(gpus, argv):
        seen["torch_loaded_by_bench"] = "torch" in bench.__dict__
        seen["args"] = (gpus, list(argv))
        return 0

    monkeypatch.setattr(bench, "launch_ranks", fake_launch)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    assert seen["args"] == (2, ["--gpus", "2", "--steps", "1"])
    assert not seen["torch_loaded_by_bench"]


def test_hw_queues_recorded(monkeypatch):
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    assert bench.hw_queues_setting() == 8 and os.environ["GPU_MAX_HW_QUEUES"] == "8"
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "16")
    assert bench.hw_queues_setting() == 16


def test_c3_streams_get_queues():
    # configs[2] on one GPU runs twelve streams in flight: 32 hardware queues before any HIP
    # call (streams beyond the queues serialize), never lowered below an explicit setting
    import types
    a = types.SimpleNamespace(config="c3", path="put", gpus=1)
    assert bench.c3_streams(a)
    assert not bench.c3_streams(types.SimpleNamespace(config="c3", path="put", gpus=8))
    assert not bench.c3_streams(types.SimpleNamespace(config="c2", path="put", gpus=1))
    assert bench.C3_QUEUES <= 32  # the GPU pool refuses more


def test_c3_queue_setting(monkeypatch):
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    assert bench.hw_queues_setting(bench.C3_QUEUES) == 32
    assert os.environ["GPU_MAX_HW_QUEUES"] == "32"
