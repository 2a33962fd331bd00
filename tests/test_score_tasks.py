"""K2 task lists (ghostm_amd/csrc/score_tasks.h, host code): compiled with g++
and checked on random candidate counts and segment cuts — every candidate in
exactly one task, each task's candidates belong to the query profiles it
builds (two ranges for the unit-pair kernel, consecutive runs otherwise),
at most one workgroup of candidates per task, and the block count used to
choose the kernel equals the built tasks'. The device side runs them in the
GPU parity tests (GHOSTM_K2=unit with GHOSTM_K2_TASKS=paired|consecutive)."""
import os
import subprocess


def test_score_tasks(tmp_path):
    src = os.path.join(os.path.dirname(__file__), "native", "test_score_tasks.cpp")
    exe = str(tmp_path / "test_score_tasks")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", src, "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "trials ok" in r.stdout
