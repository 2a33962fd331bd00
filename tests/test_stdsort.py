"""The device merge reproduces libstdc++'s std::sort permutation (the reference's
merge order, aligner.cpp:702/745, is that of an unstable introsort). The emulation
header is compiled for the host here and compared with the real std::sort on
tie-heavy random inputs; the device build of the same header is covered by the GPU
parity tests."""
import os
import subprocess


def test_stdsort_emulation_matches_libstdcxx(tmp_path):
    src = os.path.join(os.path.dirname(__file__), "native", "test_stdsort.cpp")
    exe = str(tmp_path / "test_stdsort")
    subprocess.run(["g++", "-O2", "-std=c++17", src, "-o", exe], check=True)
    r = subprocess.run([exe, "60000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout
