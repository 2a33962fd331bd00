"""`ghostm db` / `ghostm qry` (the formats the hot path reads) are byte-identical
to the reference formatters (db_creator.cpp, query_creator.cpp): every formatted
file of every dataset matches the sha256 recorded from the reference program."""
import os

import pytest

import cases

NAMES = [n for n in cases.DATASETS]


@pytest.mark.parametrize("name", NAMES)
def test_formatted_files_match_reference(name, dataset, golden):
    d = dataset(name)
    want = golden["formatted"][name]
    have = {f: cases.sha256(os.path.join(d, f)) for f in cases.formatted_files(d)}
    assert sorted(have) == sorted(want)
    for f in want:
        assert have[f] == want[f], f


def test_index_structure(dataset):
    """CSR index invariants (db_creator.cpp:167-241): ascending positions per key,
    no X-containing or END-straddling k-mer, key = 5-bit codes first residue
    most significant."""
    import numpy as np

    d = dataset("syn_small")
    seq = np.fromfile(os.path.join(d, "db_0.seq"), dtype=np.uint8)
    raw = np.fromfile(os.path.join(d, "db_0.ind"), dtype="<u4")
    seed, kcl, npos = raw[:3]
    kc = raw[3:3 + kcl]
    pos = raw[3 + kcl:3 + kcl + npos]
    assert seed == 15 and kcl == 32 ** 4 + 1 and kc[-1] == npos
    keys = np.repeat(np.arange(kcl - 1, dtype=np.int64), np.diff(kc))
    win = np.stack([seq[pos + t] for t in range(4)], axis=1).astype(np.int64)
    assert not np.any(win == 23) and not np.any(win == 25)
    recon = (win[:, 0] << 15) | (win[:, 1] << 10) | (win[:, 2] << 5) | win[:, 3]
    assert np.array_equal(recon, keys)
    order = keys * (1 << 32) + pos
    assert np.all(np.diff(order) > 0)


def test_dna_six_frames(dataset):
    """qry -t d: six frames per read, named like the read, '*'-padded."""
    import numpy as np

    d = dataset("syn_dna")
    names = open(os.path.join(d, "q_0.nam")).read().splitlines()
    assert len(names) == 6 * 300
    assert all(names[6 * i + k] == names[6 * i] for i in range(300) for k in range(6))
    L = int(np.fromfile(os.path.join(d, "q_0.inf"), dtype="<u4")[1])
    assert L == 50
