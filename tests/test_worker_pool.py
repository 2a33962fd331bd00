"""The host thread pool behind ParallelFor (text formatting, file loads):
concurrent and nested jobs and exceptions, under ThreadSanitizer."""
import os
import subprocess

HERE = os.path.dirname(__file__)
CSRC = os.path.join(os.path.dirname(HERE), "ghostm_amd", "csrc")


def test_worker_pool_tsan(tmp_path):
    exe = str(tmp_path / "test_worker_pool")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=thread", "-I", CSRC,
                    os.path.join(HERE, "native", "test_worker_pool.cpp"), "-o", exe, "-pthread"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr
