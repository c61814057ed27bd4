"""--profile (utils/profiling.py): the parent re-runs the entry point under rocprofv3 as ONE child
process, without --profile, and summarises the kernel stats; the child runs normally."""
import os
import sys

import pytest

from fraud_detection_spark_kafka_llm_amd.utils import profiling


def test_child_command_puts_the_program_right_after_the_separator(tmp_path):
    cmd = profiling.child_command(["--steps", "3", "--profile", "--gpus", "1"], str(tmp_path), rocprof="/x/rocprofv3")
    assert cmd[:6] == ["/x/rocprofv3", "--kernel-trace", "--stats", "-d", str(tmp_path), "-o"]
    sep = cmd.index("--")
    assert cmd[sep + 1] == sys.executable           # no shell / env hop after "--"
    assert "--profile" not in cmd and cmd[-4:] == ["--steps", "3", "--gpus", "1"]
    mod = profiling.child_command([], str(tmp_path), module="fraud_detection_spark_kafka_llm_amd.train",
                                  rocprof="/x/rocprofv3")
    assert mod[mod.index("--") + 1:] == [sys.executable, "-m", "fraud_detection_spark_kafka_llm_amd.train"]


def test_parent_runs_one_child_and_exits_with_its_status(tmp_path, monkeypatch):
    calls = []
    stats = tmp_path / "host" / "run_kernel_stats.csv"
    stats.parent.mkdir()
    stats.write_text('"Name","Calls","TotalDurationNs","AverageNs","Percentage"\n'
                     '"hist_i8_kernel",10,5000000,500000,80.0\n"split_kernel",10,1000000,100000,20.0\n')

    def fake_call(cmd, env):
        calls.append((cmd, env))
        return 3

    monkeypatch.delenv(profiling.CHILD_ENV, raising=False)
    monkeypatch.setattr(profiling.subprocess, "call", fake_call)
    monkeypatch.setattr(profiling.shutil, "which", lambda name: "/bin/true")
    with pytest.raises(SystemExit) as e:
        profiling.run_profiled_if_requested(True, ["--profile", "--steps", "2"], out_dir=str(tmp_path))
    assert e.value.code == 3 and len(calls) == 1
    cmd, env = calls[0]
    assert env[profiling.CHILD_ENV] == "1" and "--profile" not in cmd
    assert profiling.kernel_stats(str(tmp_path))[0][:3] == ("hist_i8_kernel", 10, 5.0)
    # in the child (or without --profile) it is a no-op
    monkeypatch.setenv(profiling.CHILD_ENV, "1")
    profiling.run_profiled_if_requested(True, ["--profile"], out_dir=str(tmp_path))
    monkeypatch.delenv(profiling.CHILD_ENV)
    profiling.run_profiled_if_requested(False, [], out_dir=str(tmp_path))
    assert len(calls) == 1
