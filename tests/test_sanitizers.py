"""SURVEY §5.2 race/memory checking on the host paths: the multi-threaded CPU featurizer (hashing
and token-key modes), JSON extraction and tree engine run under AddressSanitizer +
UndefinedBehaviorSanitizer in a standalone build (csrc/tests/host_selftest.cpp)."""
import os
import shutil
import subprocess

import pytest

from fraud_detection_spark_kafka_llm_amd import _build


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs hipcc")
def test_host_paths_clean_under_asan_ubsan():
    exe = _build.build_host_selftest(sanitize=True)
    res = subprocess.run([str(exe)], env={**os.environ, **_build.SELFTEST_ENV}, capture_output=True, text=True,
                         timeout=300)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "host selftest OK" in res.stdout
    assert "runtime error" not in res.stderr      # UBSan diagnostics
