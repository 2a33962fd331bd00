"""The multi-GPU data path exactly as the driver's 8-GPU run executes it, at
world 1 on one MI355X.

bench.py is started as a rank of its own (RANK/WORLD_SIZE/LOCAL_RANK and
MASTER_* in the environment, as torchrun or `bench.py --gpus N` sets them) with
GHOSTM_BENCH_DIST=1, so it takes the collective path at world 1: RCCL
(backend "nccl") process group bound to the device, NUMA placement of every
thread, the per-step ok-flag agreement on cuda tensors, the gather buffer
filled device to device by GhostmSessionDeviceHits (`device_hits_into`), the
RCCL gather, and rank 0's check of the gathered records and the assembled
file against an unsharded run. The gloo rehearsals take the other fill branch;
this test is the one that runs the RCCL branch."""
import json
import os
import re
import subprocess
import sys

import pytest

from ghostm_amd.launch import free_port

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_rccl_data_path_world1(tmp_path):
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", LOCAL_WORLD_SIZE="1", GROUP_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), GHOSTM_BENCH_DIST="1",
               GHOSTM_BENCH_PG_TIMEOUT="120")
    env.pop("GHOSTM_BENCH_BACKEND", None)
    env.pop("GHOSTM_BENCH_NO_BIND", None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--preset", "cfg4", "--queries", "20000",
           "--steps", "2", "--warmup", "1", "--no-cpu", "--workdir", str(tmp_path)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout  # stdout carries only rank 0's JSON line
    line = json.loads(lines[0])
    out = os.environ.get("GHOSTM_TEST_OUT")
    if out:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "bench_rccl_world1.json"), "w") as f:
            f.write(lines[0] + "\n")
    assert line["value"] and line["ranks"] == 1
    # the gather ran over RCCL with the device-to-device fill in every step
    fill = line["gather_fill"]
    assert fill["backend"] == "nccl"
    assert fill["device_hits_into"] == 3 and fill["device_hits_copy"] == 0  # 1 warmup + 2 timed
    chk = line["gather_check"]
    assert chk["records_gathered"] > 0
    assert all(v for k, v in chk.items() if k != "records_gathered"), chk
    assert line["output_matches_unsharded_run"] is True
    assert line["end_to_end"]["output_files_match_timed_run"] is True
    # placement on the GPU's own PCI address, every thread bound
    pl = line["per_rank"][0]["placement"]
    assert re.fullmatch(r"[0-9a-f]{4}:[0-9a-f]{2}:[0-9a-f]{2}\.0", pl["pci"]), pl
    assert pl["bound"] is True and pl["threads_bound"] >= 1, pl
