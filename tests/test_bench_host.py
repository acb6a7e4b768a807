"""bench.py host logic (no GPU): the multi-GPU launcher and the roofline
arithmetic of SURVEY §8(d)."""
import os
import subprocess
import sys

import pytest

import bench


def test_launcher_command_runs_torchrun_as_child():
    cmd = bench.launcher_command(["--gpus", "2", "--steps", "3"], 2, port=29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and "--master-port=29511" in cmd
    assert cmd[cmd.index("--master-port=29511") + 1] == os.path.abspath(bench.__file__)
    assert cmd[-4:] == ["--gpus", "2", "--steps", "3"]


def test_gpus_flag_spawns_ranks_without_touching_the_gpu(monkeypatch):
    """`bench.py --gpus 4` outside torchrun starts the rank launcher as a
    subprocess and exits with its return code (never an exec)."""
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    import torch
    monkeypatch.setattr(torch.cuda, "set_device", lambda *a: pytest.fail("touched the GPU"))
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7
    assert "--nproc-per-node=4" in seen["cmd"] and seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_encode_bytes_per_image_matches_survey():
    # 3,591,168 B per 512^2 image, 713,472 B per 224^2 image
    assert bench.encode_bytes_per_image(512, 512, 3072, 14, 3072, 1) == 3591168
    assert bench.encode_bytes_per_image(224, 224, 768, 14, 3072, 4) == 713472
