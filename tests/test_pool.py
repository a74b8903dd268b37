"""The host worker pool behind the library's parallel_for / parallel_tasks (csrc/common.hpp
WorkerPool): tests/pool_check.cpp compiled against the header and run on the CPU (no GPU calls)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "large-scale-recommendation_amd", "csrc")


def test_worker_pool(tmp_path):
    cxx = shutil.which("g++")
    if cxx is None or not os.path.isdir("/opt/rocm/include"):
        pytest.skip("no g++ or ROCm headers")
    exe = tmp_path / "pool_check"
    cmd = [cxx, "-O1", "-std=c++17", "-pthread", "-D__HIP_PLATFORM_AMD__", "-I", CSRC,
           "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
           os.path.join(ROOT, "tests", "pool_check.cpp"), "-o", str(exe),
           "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, MFHIP_THREADS="8")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and r.stdout.strip() == "ok", (r.stdout, r.stderr)
