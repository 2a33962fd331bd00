"""The formatter's host buffers (host_buffers.h: TextBuf, HostAllocator,
HostAlloc), under AddressSanitizer on the host."""
import os
import subprocess

HERE = os.path.dirname(__file__)
CSRC = os.path.join(os.path.dirname(HERE), "ghostm_amd", "csrc")


def test_host_buffers_asan(tmp_path):
    exe = str(tmp_path / "test_host_buffers")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-I", CSRC,
                    os.path.join(HERE, "native", "test_host_buffers.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
