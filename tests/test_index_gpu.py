"""GPU k-mer index build (include/ghostm_hip.h GhostmBuildIndexGpu,
replacing DBCreator::ConstructIndex, db_creator.cpp:167-241).

`ghostm db -D 0` must write the same bytes as the CPU formatter, whose files are
pinned to the reference program by tests/test_formatter.py. Spaced seeds (not
reachable from the CLI) are checked through the C ABI against a numpy
restatement of ConstructIndex."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import cases

pytestmark = pytest.mark.gpu

EDGE_FASTA = """>exact4
ACDE
>short3
WYV
>five
ACDEF
>with_x
ACDXEFGHIKXLMNPQ
>lower
acdefghiklmnpqrstvwy
>ambig
BZJUOACDEFGHBZ
>x_edges
XACDEFX
>long
MKTAYIAKQRQISFVKSHFSRQLEERLGLIEVQAPILSRVGDGTQDNLSGAEKAVQVKVKALPDAQFEVVHSLAKWKRQTLGQHDFSAGEGLYTHMKALRPDEDRLSPLHSVYVDQWDWERVMGDGERQFSTLKSTVEAIWAGIKATEAAVSEEFGLAPFLPDQIHFVHSQELLSRYPDLDAKGRERAIAKDLGAVFLVGIGGKLSDGHRHDVRAPDYDDWUAIGLNEVEVRH
>e1
A
>tail4
MKTA
"""


def _db_files(d, prefix):
    return sorted(f for f in os.listdir(d) if f.startswith(prefix + "_") or f == prefix + ".inf")


@pytest.mark.parametrize("name", ["protein_testset", "readme_kat", "syn_small", "syn_short", "syn_chunks"])
def test_db_gpu_index_matches_cpu(name, dataset, tmp_path):
    """Every chunk's .ind from `db -D 0` equals the CPU formatter's (k=4; syn_short
    k=3; syn_chunks 3 chunks)."""
    d = dataset(name)
    _, args = [t for t in cases.DATASETS[name] if t[0] == "db"][0]
    a = [x.format(d=d, golden=cases.GOLDEN) for x in args]
    a[a.index("-o") + 1] = str(tmp_path / "db")
    subprocess.run([cases.GHOSTM, "db"] + a + ["-D", "0"], check=True, capture_output=True)
    want = _db_files(d, "db")
    have = _db_files(str(tmp_path), "db")
    assert want == have
    for f in want:
        assert cases.sha256(os.path.join(d, f)) == cases.sha256(os.path.join(str(tmp_path), f)), f


@pytest.mark.parametrize("k", ["4", "3", "2", "5"])
def test_db_gpu_index_edge_subjects(k, tmp_path):
    """Subjects of exactly the seed span (skipped by the reference), shorter ones,
    X inside and at the edges, lower case, ambiguous letters, a one-residue tail."""
    fa = tmp_path / "edge.fa"
    fa.write_text(EDGE_FASTA)
    for dev, out in ((None, "cpu"), ("0", "gpu")):
        cmd = [cases.GHOSTM, "db", "-i", str(fa), "-o", str(tmp_path / out), "-k", k]
        if dev is not None:
            cmd += ["-D", dev]
        subprocess.run(cmd, check=True, capture_output=True)
    for suffix in (".ind", ".seq", ".pos", ".inf", ".nam"):
        a = (tmp_path / ("cpu_0" + suffix)).read_bytes()
        b = (tmp_path / ("gpu_0" + suffix)).read_bytes()
        assert a == b, suffix


def _restated_index(seq: np.ndarray, seed: int):
    """ConstructIndex (db_creator.cpp:183-233) in numpy: per subject longer than the
    span, windows without X/END, key over the seed's set positions."""
    span = seed.bit_length()
    weight = bin(seed).count("1")
    kcl = 32 ** weight + 1
    ends = np.flatnonzero(seq == 25)
    starts = np.concatenate([[0], ends[:-1] + 1])
    keys, pos = [], []
    for s, e in zip(starts, ends):
        if e - s <= span:
            continue
        for j in range(s, e - span + 1):
            w = seq[j:j + span]
            if np.any(w == 23):
                continue
            key = 0
            for t in range(span):
                if (seed >> t) & 1:
                    key = (key << 5) | int(w[t])
            keys.append(key)
            pos.append(j)
    keys = np.asarray(keys, dtype=np.int64)
    pos = np.asarray(pos, dtype=np.uint32)
    order = np.lexsort((pos, keys))
    kc = np.zeros(kcl, dtype=np.uint32)
    np.add.at(kc, keys + 1, 1)
    return np.cumsum(kc, dtype=np.uint32), pos[order]


@pytest.mark.parametrize("seed", [0b1011, 0b11011, 0b111, 0b1])
def test_spaced_seed_index_matches_restatement(seed, dataset):
    from ghostm_amd.native import load, last_error

    d = dataset("syn_small")
    seq = np.fromfile(os.path.join(d, "db_0.seq"), dtype=np.uint8)[:60000].copy()
    seq[-1] = 25  # a chunk ends with an END
    want_kc, want_pos = _restated_index(seq, seed)
    lib = load()
    kcl = 32 ** bin(seed).count("1") + 1
    kc = np.zeros(kcl, dtype=np.uint32)
    pos = np.zeros(len(seq), dtype=np.uint32)
    npos = ctypes.c_uint32(0)
    ms = ctypes.c_float(0)
    u32 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))  # noqa: E731
    rc = lib.GhostmBuildIndexGpu(seq.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), len(seq), seed, kcl,
                                 u32(kc), u32(pos), ctypes.byref(npos), 0, ctypes.byref(ms))
    assert rc == 0, last_error()
    assert np.array_equal(kc, want_kc)
    assert npos.value == len(want_pos)
    assert np.array_equal(pos[:npos.value], want_pos)


def test_index_abi_errors():
    from ghostm_amd.native import load, last_error

    lib = load()
    seq = np.array([0, 1, 2, 3, 4, 25], dtype=np.uint8)
    kc = np.zeros(32 ** 4 + 1, dtype=np.uint32)
    pos = np.zeros(6, dtype=np.uint32)
    npos = ctypes.c_uint32(0)
    u32 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))  # noqa: E731
    p8 = seq.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
    # wrong keys_count length for the seed
    assert lib.GhostmBuildIndexGpu(p8, 6, 15, 100, u32(kc), u32(pos), ctypes.byref(npos), 0, None) != 0
    assert "keys_count" in last_error()
    assert lib.GhostmBuildIndexGpu(p8, 6, 15, 32 ** 4 + 1, u32(kc), u32(pos), ctypes.byref(npos), 0, None) == 0
    assert npos.value == 2 and kc[-1] == 2


def _restated_index_solid(seq: np.ndarray, span: int = 4):
    """Vectorised ConstructIndex for a solid seed of `span` ones (the rule of
    _restated_index, db_creator.cpp:183-233), for sizes the loop is too slow for."""
    n = len(seq)
    kcl = 32 ** span + 1
    m = n - span  # windows with j + span < n (the chunk ends with an END)
    if m <= 0:
        return np.zeros(kcl, dtype=np.uint32), np.zeros(0, dtype=np.uint32)
    bad = ((seq == 25) | (seq == 23)).astype(np.int32)
    cb = np.concatenate([[0], np.cumsum(bad)])
    j = np.arange(m)
    ok = (cb[j + span] - cb[j]) == 0
    starts_subject = (j == 0) | (seq[np.maximum(j - 1, 0)] == 25)
    ok &= ~(starts_subject & (seq[j + span] == 25))
    keys = np.zeros(m, dtype=np.int64)
    for t in range(span):
        keys = (keys << 5) | seq[j + t].astype(np.int64)
    keys, pos = keys[ok], j[ok].astype(np.uint32)
    order = np.argsort(keys, kind="stable")
    kc = np.zeros(kcl, dtype=np.uint32)
    np.add.at(kc, keys + 1, 1)
    return np.cumsum(kc, dtype=np.uint32), pos[order]


@pytest.mark.parametrize("n", [2, 65, 4095, 4096, 4097, 8193, 250001])
def test_index_radix_sort_tile_edges(n):
    """The hand-written radix sort (index.hip k_rs_*) at lengths around its
    4096-element tiles and 64-element batches: CSR and positions equal a numpy
    stable sort of the same windows."""
    from ghostm_amd.native import load, last_error

    rng = np.random.default_rng(n)
    seq = rng.integers(0, 23, size=n).astype(np.uint8)
    seq[rng.random(n) < 0.004] = 23  # X
    seq[rng.random(n) < 0.01] = 25   # subject ends
    seq[-1] = 25
    want_kc, want_pos = _restated_index_solid(seq)
    lib = load()
    kcl = 32 ** 4 + 1
    kc = np.zeros(kcl, dtype=np.uint32)
    pos = np.zeros(n, dtype=np.uint32)
    npos = ctypes.c_uint32(0)
    u32 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))  # noqa: E731
    rc = lib.GhostmBuildIndexGpu(seq.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), n, 0b1111, kcl,
                                 u32(kc), u32(pos), ctypes.byref(npos), 0, None)
    assert rc == 0, last_error()
    assert np.array_equal(kc, want_kc)
    assert npos.value == len(want_pos)
    assert np.array_equal(pos[:npos.value], want_pos)
