"""Uninitialised-LDS reads made deterministic.

Round 4 found a stale-LDS read (an invalid half of a paired K2 task reading a
slot-1 profile word no block had written) only because the stale value
happened to differ on one run. The poison build (make -C ghostm_amd/csrc:
ghostm_amd/lib/libghostm_hip_poison.so, -DGHOSTM_LDS_POISON=1) has every kernel
fill its whole LDS allocation — static and dynamic, the dispatch packet's
group_segment_size — with a pattern before its own code runs. Any read of LDS
the kernel did not write then returns that pattern: if a result depended on
it, the output differs from the reference's under at least one of two
patterns. Each (pattern, group) runs in one child process that loads the
poison build through GHOSTM_LIB_PATH (tests/lds_poison_child.py)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
POISON_LIB = os.path.join(os.path.dirname(HERE), "ghostm_amd", "lib", "libghostm_hip_poison.so")


@pytest.mark.parametrize("group", ["golden", "kernels"])
@pytest.mark.parametrize("pattern", ["0xA5A5A5A5", "0x00000000"])
def test_golden_variants_under_lds_poison(pattern, group, data_root):
    assert os.path.exists(POISON_LIB), "build the poison library (make -C ghostm_amd/csrc)"
    env = dict(os.environ, GHOSTM_LIB_PATH=POISON_LIB, GHOSTM_LDS_POISON_PATTERN=pattern)
    p = subprocess.run([sys.executable, os.path.join(HERE, "lds_poison_child.py"), group, data_root],
                       capture_output=True, text=True, timeout=115, env=env)
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert lines, p.stderr[-3000:]
    res = json.loads(lines[-1])
    assert p.returncode == 0 and not res.get("failures") and not res.get("error"), res
    assert res["runs"] >= (176 if group == "golden" else 50)
