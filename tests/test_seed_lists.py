"""K1 phase 0's entry -> list byte table (ghostm_amd/csrc/seed_lists.h, shared
with k_seed_filter): compiled with g++ and checked against a per-entry walk over
the list offsets on random list sets (empty lists, boundaries at every position
of a 16-entry window). The kernel itself runs in the GPU parity tests."""
import os
import subprocess


def test_seed_list_bytes(tmp_path):
    src = os.path.join(os.path.dirname(__file__), "native", "test_seed_lists.cpp")
    exe = str(tmp_path / "test_seed_lists")
    subprocess.run(["g++", "-O2", "-std=c++17", src, "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "trials ok" in r.stdout


def _table_buckets():
    """kBuckets (= TSLOTS / 4) of every BinTable the library instantiates: the
    k_seed_hash launches and the k_seed_filter classes in device.hip."""
    import re

    src = open(os.path.join(os.path.dirname(__file__), "..", "ghostm_amd", "csrc", "device.hip")).read()
    tslots = {int(m) for m in re.findall(r"k_seed_hash<\d+, (\d+)>", src)}
    tslots |= {int(m) for m in re.findall(r"#define GHOSTM_FILTER\d kern::k_seed_filter<\d+, [^,]+, (\d+),", src)}
    return sorted(t // 4 for t in tslots)


def test_bin_table_buckets_in_range(tmp_path):
    """Every bucket of K1's bin table hash is inside its table for every bin
    <= kHashBinLimit + 1 and every instantiated table size (the round-5 hang's
    cause: an arithmetic shift put buckets outside the table, and the probe
    loop never ended). The signed-shift form is the negative control."""
    buckets = _table_buckets()
    assert len(buckets) >= 6, buckets  # three hash classes, three filter classes
    src = os.path.join(os.path.dirname(__file__), "native", "test_bin_bucket.cpp")
    exe = str(tmp_path / "test_bin_bucket")
    subprocess.run(["g++", "-O2", "-std=c++17", f"-DBUCKETS={','.join(map(str, buckets))}", src, "-o", exe],
                   check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all buckets in range" in r.stdout
