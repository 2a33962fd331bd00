"""GPU parity: the HIP path (through the C ABI) against the oracle and the reference
golden outputs. Bit-exact text for every dataset/option variant; stage-level checks
of the reference plugin surface (SearchNextGpu / CalculateScoreGpu / TraceBackGpu)
against the oracle's stage dumps."""
import ctypes
import os

import numpy as np
import pytest

import cases
from ghostm_amd import native
from ghostm_amd.aligner import Session

pytestmark = pytest.mark.gpu


def _gpu_text(d, opts, env, out):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        with Session(["-i", os.path.join(d, "q"), "-d", os.path.join(d, "db"), "-o", out, "-D", "0"]
                     + list(opts)) as s:
            s.run()
            text = s.output()
            st = s.stats()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return text, st


@pytest.mark.parametrize("ds,var,opts,env", cases.VARIANTS, ids=[f"{v[0]}/{v[1]}" for v in cases.VARIANTS])
def test_gpu_matches_reference_golden(ds, var, opts, env, dataset, golden, tmp_path):
    d = dataset(ds)
    text, st = _gpu_text(d, opts, env, str(tmp_path / "g.out"))
    want = golden["aln"][f"{ds}/{var}"]
    (tmp_path / "g.out").write_bytes(text)
    assert text.count(b"\n") == want["lines"]
    assert cases.sha256(str(tmp_path / "g.out")) == want["sha256"]


@pytest.mark.parametrize("tasks", ["paired", "consecutive"])
@pytest.mark.parametrize("ds,var,opts,env", cases.VARIANTS, ids=[f"{v[0]}/{v[1]}" for v in cases.VARIANTS])
def test_gpu_unit_k2_matches_reference_golden(ds, var, opts, env, tasks, dataset, golden, tmp_path):
    """Every golden variant with K2's unit-pair kernel forced (GHOSTM_K2=unit;
    by default it runs only on segments averaging enough candidates per
    query), with its tasks as query pairs (two candidate ranges per block) or
    as consecutive runs: windows crossing one or several subject ENDs (the
    testset's short subjects), a window whose first column is END, the DB's
    end, one-subject DBs, short queries (S = 16 and 8) and every gap setting."""
    d = dataset(ds)
    text, st = _gpu_text(d, opts, dict(env, GHOSTM_K2="unit", GHOSTM_K2_TASKS=tasks), str(tmp_path / "g.out"))
    want = golden["aln"][f"{ds}/{var}"]
    (tmp_path / "g.out").write_bytes(text)
    assert cases.sha256(str(tmp_path / "g.out")) == want["sha256"]
    if st["score_launches_swar"] == st["score_launches"] > 0:  # integer patterns fit: the unit kernel ran
        assert st["score_launches_unit"] == st["score_launches"]


@pytest.mark.parametrize("ds,var,opts,env", cases.VARIANTS, ids=[f"{v[0]}/{v[1]}" for v in cases.VARIANTS])
def test_gpu_pair_k2_matches_reference_golden(ds, var, opts, env, dataset, golden, tmp_path):
    """Every golden variant with the pair-table K2 forced at any density
    (GHOSTM_K2=pair: k_score_pair; by default sparse segments, fewer than
    kScorePairMax = 16 candidates per query, run the sparse rows kernel and
    GHOSTM_K2_SPARSE=pair selects this one): windows over one or several
    subject ENDs, a window starting at an END, the DB's end, one-subject DBs,
    S = 16 and 8, G = 1, odd candidate counts (single pairs), every gap setting."""
    d = dataset(ds)
    text, st = _gpu_text(d, opts, dict(env, GHOSTM_K2="pair"), str(tmp_path / "g.out"))
    want = golden["aln"][f"{ds}/{var}"]
    (tmp_path / "g.out").write_bytes(text)
    assert cases.sha256(str(tmp_path / "g.out")) == want["sha256"]
    if st["score_launches_swar"] == st["score_launches"] > 0:  # integer patterns fit: the pair kernel ran
        assert st["score_launches_pair"] == st["score_launches"]


@pytest.mark.parametrize("ds,var,opts,env", cases.VARIANTS, ids=[f"{v[0]}/{v[1]}" for v in cases.VARIANTS])
def test_gpu_sparse_rows_k2_matches_reference_golden(ds, var, opts, env, dataset, golden, tmp_path):
    """Every golden variant with the sparse segments' 16-row profile kernel forced
    at any density (GHOSTM_K2=sparse: k_score16f<16, true> with seven 27-row query
    profiles per block, kScoreRowsSparse): the same windows, ENDs, DB ends,
    short queries and gap settings as the other K2 forms."""
    d = dataset(ds)
    text, st = _gpu_text(d, opts, dict(env, GHOSTM_K2="sparse"), str(tmp_path / "g.out"))
    want = golden["aln"][f"{ds}/{var}"]
    (tmp_path / "g.out").write_bytes(text)
    assert cases.sha256(str(tmp_path / "g.out")) == want["sha256"]
    if st["score_launches_swar"] == st["score_launches"] > 0:  # integer patterns fit: the sparse kernel ran
        assert st["score_launches_sparse"] == st["score_launches"]


@pytest.mark.parametrize("form", ["default", "sparse", "swar16", "levels0", "sparse_levels0"])
@pytest.mark.parametrize("ds,var,opts", [("syn_subj10", "default", []), ("syn_subj10", "y2", ["-y", "2"]),
                                         ("syn_subj4", "default", []), ("protein_testset", "y0", []),
                                         ("cfg2_single", "default", [])])
def test_k2_restart_levels_match_golden(form, ds, var, opts, dataset, golden, tmp_path):
    """K2's restart levels (k_score16f<S, true, false, true>: each END of a
    window restarts one level higher, E floored at the level in the column
    before, no second-END reset) on DBs whose windows cross many subject ENDs
    (10-20-residue subjects: up to 15 per window), against the oracle; with
    4-9-residue subjects the levels do not fit and the reset kernel runs
    instead. GHOSTM_K2_LEVELS=0 forces the reset kernel everywhere. Against the
    reference program's output (golden) and the oracle."""
    d = dataset(ds)
    env = {"sparse": {"GHOSTM_K2": "sparse"}, "swar16": {"GHOSTM_K2": "swar16"},
           "levels0": {"GHOSTM_K2": "swar16", "GHOSTM_K2_LEVELS": "0"},
           "sparse_levels0": {"GHOSTM_K2": "sparse", "GHOSTM_K2_LEVELS": "0"}}.get(form, {})
    text, st = _gpu_text(d, opts, env, str(tmp_path / "g.out"))
    (tmp_path / "g.out").write_bytes(text)
    assert cases.sha256(str(tmp_path / "g.out")) == golden["aln"][f"{ds}/{var}"]["sha256"]
    assert text == cases.run_aln(cases.ORACLE, d, opts, {}, str(tmp_path / "o.out"))
    assert text.count(b"\n") > (50 if ds.startswith("syn_subj") else 0)
    assert st["score_launches_swar"] == st["score_launches"] > 0
    rows = st["score_launches"] - st["score_launches_unit"] - st["score_launches_pair"]
    if form in ("levels0", "sparse_levels0") or ds == "syn_subj4":
        assert st["score_launches_levels"] == 0
    elif form != "default":  # the forced 16-bit-row kernels, with levels
        assert st["score_launches_levels"] == rows == st["score_launches"]
    else:
        assert st["score_launches_levels"] == rows


@pytest.mark.parametrize("merge", ["device", "device_thread", "host"])
@pytest.mark.parametrize("ds,var,opts,env", cases.BATCH_VARIANTS,
                         ids=[f"{v[0]}/{v[1]}" for v in cases.BATCH_VARIANTS])
def test_gpu_batch_cuts_match_oracle(merge, ds, var, opts, env, dataset, tmp_path):
    """CPU-path batch semantics (carry, drop of a carried last query, stop at the
    first empty batch) at tiny -l, against the oracle: on the device (K4 merges
    every batch's candidates with the carried result lists, wave and one-thread
    kernels) and with the host merge (GHOSTM_MERGE=host)."""
    d = dataset(ds)
    env = dict(env)
    if merge == "host":
        env["GHOSTM_MERGE"] = "host"
    elif merge == "device_thread":
        env["GHOSTM_K4"] = "thread"
    text, st = _gpu_text(d, opts, env, str(tmp_path / "g.out"))
    want = cases.run_aln(cases.ORACLE, d, opts, {k: v for k, v in env.items() if k.startswith("GHOSTM_MAX")},
                         str(tmp_path / "o.out"))
    assert text == want
    if env.get("GHOSTM_MAX_LIST_OVERRIDE") not in ("1",):
        assert st["batches"] > 1
    if merge == "host" or st["batches"] == 0:
        assert st["merge_launches"] == 0
    else:
        assert st["merge_launches"] > 0


@pytest.mark.parametrize("merge", ["device", "host"])
@pytest.mark.parametrize("var,opts", [("default", []), ("b20_y2", ["-b", "20", "-y", "2"]), ("S1", ["-S", "1"])])
def test_multi_db_chunk_merge(merge, var, opts, dataset, golden, tmp_path):
    """Three DB chunks: the result lists carried from chunk to chunk are merged
    on the device (K4) or on the host, both equal to the reference."""
    d = dataset("syn_chunks")
    env = {"GHOSTM_MERGE": "host"} if merge == "host" else {}
    text, st = _gpu_text(d, opts, env, str(tmp_path / "g.out"))
    (tmp_path / "g.out").write_bytes(text)
    assert cases.sha256(str(tmp_path / "g.out")) == golden["aln"][f"syn_chunks/{var}"]["sha256"]
    assert (st["merge_launches"] == 0) if merge == "host" else (st["merge_launches"] > 0)


def test_cli_aln_writes_same_file(dataset, golden, tmp_path):
    d = dataset("syn_small")
    out = tmp_path / "cli.out"
    cases.run_aln(cases.GHOSTM, d, ["-D", "0"], {}, str(out))
    assert cases.sha256(str(out)) == golden["aln"]["syn_small/default"]["sha256"]


def test_session_rerun_is_identical(dataset, tmp_path):
    d = dataset("syn_small")
    with Session(["-i", f"{d}/q", "-d", f"{d}/db", "-o", str(tmp_path / "x"), "-D", "0"]) as s:
        s.run()
        a, ha = s.output(), s.hits()
        s.run()
        b, hb = s.output(), s.hits()
    assert a == b and np.array_equal(ha, hb)
    assert len(ha) == a.count(b"\n")


# ------------------------------------------------------------ stage level
def _load_chunk(d, qprefix="q", dprefix="db"):
    inf = np.fromfile(f"{d}/{qprefix}_0.inf", dtype="<u4")
    nq, L = int(inf[0]), int(inf[1])
    qseq = np.fromfile(f"{d}/{qprefix}_0.seq", dtype=np.uint8)
    dinf = np.fromfile(f"{d}/{dprefix}_0.inf", dtype="<u4")
    dbseq = np.fromfile(f"{d}/{dprefix}_0.seq", dtype=np.uint8)
    raw = np.fromfile(f"{d}/{dprefix}_0.ind", dtype="<u4")
    seed, kcl, npos = (int(x) for x in raw[:3])
    kc = np.ascontiguousarray(raw[3:3 + kcl])
    pos = np.ascontiguousarray(raw[3 + kcl:3 + kcl + npos])
    assert len(dbseq) == int(dinf[1])
    return nq, L, qseq, dbseq, seed, kc, pos


def _p(a, t=ctypes.c_uint32):
    return a.ctypes.data_as(ctypes.POINTER(t))


def _blosum62():
    return cases.parse_ncbi_matrix(os.path.join(cases.GOLDEN, "matrices", "BLOSUM62"))


@pytest.mark.parametrize("ds", ["syn_small", "readme_kat"])
def test_reference_abi_stages_match_oracle(ds, dataset, tmp_path):
    """InitGpu/SetOptionGpu/SetQueryGpu/SetDbGpu/SearchNextGpu/CalculateScoreGpu in
    the order the reference aligner.cpp drives them, then TraceBackGpu, compared
    with the oracle's per-candidate (start, score, end) and traceback dumps.
    readme_kat (L = 25) runs the one-lane-per-candidate layout (G = 1)."""
    d = dataset(ds)
    prefix = str(tmp_path / "dump")
    cases.run_aln(cases.ORACLE, d, ["-y", "1"], {"GHOSTM_ORACLE_DUMP": prefix}, str(tmp_path / "o"))
    cand = np.fromfile(prefix + ".cand", dtype="<u4").reshape(-1, 4)
    tb = np.fromfile(prefix + ".tb", dtype="<u4").reshape(-1, 5)

    nq, L, qseq, dbseq, seed, kc, pos = _load_chunk(d)
    lib = native.load()
    m = _blosum62()
    max_list = 1 << 27
    assert lib.InitGpu() == 0
    assert lib.SetOptionGpu(max_list, m.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), 0) == 0, native.last_error()
    assert lib.SetQueryGpu(_p(qseq, ctypes.c_uint8), nq, L) == 0, native.last_error()
    assert lib.SetDbGpu(_p(dbseq, ctypes.c_uint8), len(dbseq), _p(kc), len(kc), _p(pos), len(pos)) == 0
    acl = np.zeros(nq + 1, dtype=np.uint32)
    starts = np.zeros(len(cand) + 16, dtype=np.uint32)
    qc = lib.SearchNextGpu(L, nq, seed, 2, 2, 4, max_list, 0, _p(acl), _p(starts))
    assert qc == nq, native.last_error()
    n = int(acl[qc])
    assert n == len(cand)
    qid = np.repeat(np.arange(nq, dtype=np.uint32), np.diff(acl[: qc + 1]))
    assert np.array_equal(qid, cand[:, 0])
    assert np.array_equal(starts[:n], cand[:, 1])
    scores = np.zeros(n, dtype=np.uint32)
    ends = np.zeros(n, dtype=np.uint32)
    base = L + 2 * 2 + 2 * 16
    lib.CalculateScoreGpu(len(dbseq), L, n, _p(scores), _p(ends), base, 2, -11, -1)
    assert np.array_equal(scores, cand[:, 2])
    assert np.array_equal(ends, cand[:, 3])
    # traceback of exactly the oracle's hits
    k = len(tb)
    out_s, out_l, out_m = (np.zeros(k, dtype=np.uint32) for _ in range(3))
    out_id = np.zeros(k, dtype=np.float32)
    tqid = np.ascontiguousarray(tb[:, 0])
    tend = np.ascontiguousarray(tb[:, 1])
    rc = lib.TraceBackGpu(k, _p(tqid), _p(tend), L, L + 2 * 2 * 2 * 16, -11, -1, _p(out_s), _p(out_l),
                          _p(out_m), out_id.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    assert rc == 0, native.last_error()
    assert np.array_equal(out_s, tb[:, 2])
    assert np.array_equal(out_l, tb[:, 3])
    assert np.array_equal(out_m, tb[:, 4])
    counts = np.zeros(nq, dtype=np.uint32)
    assert lib.CountCandidatesGpu(L, nq, seed, 2, 2, 4, _p(counts)) == 0
    assert np.array_equal(counts, np.diff(acl[: qc + 1]))
    assert lib.FreeGpu() == 0


def test_reference_gpu_batching_rule(dataset):
    """SearchNextGpu batches with the reference GPU rule (aligner_gpu.cu:911-920):
    queries are added while the running total stays below max_number_alignments."""
    d = dataset("syn_small")
    nq, L, qseq, dbseq, seed, kc, pos = _load_chunk(d)
    lib = native.load()
    m = _blosum62()
    assert lib.SetOptionGpu(1 << 27, m.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), 0) == 0
    assert lib.SetQueryGpu(_p(qseq, ctypes.c_uint8), nq, L) == 0
    assert lib.SetDbGpu(_p(dbseq, ctypes.c_uint8), len(dbseq), _p(kc), len(kc), _p(pos), len(pos)) == 0
    counts = np.zeros(nq, dtype=np.uint32)
    assert lib.CountCandidatesGpu(L, nq, seed, 2, 2, 4, _p(counts)) == 0
    cap = 40
    start, seen = 0, 0
    acl = np.zeros(nq + 1, dtype=np.uint32)
    starts = np.zeros(int(counts.sum()) + 16, dtype=np.uint32)
    while True:
        qc = lib.SearchNextGpu(L, nq, seed, 2, 2, 4, cap, start, _p(acl), _p(starts))
        if qc == 0:
            break
        assert acl[qc] < cap
        assert np.array_equal(np.diff(acl[: qc + 1]), counts[start:start + qc])
        if start + qc < nq:
            assert acl[qc] + counts[start + qc] >= cap
        seen += qc
        start += qc
    assert seen == start
    lib.FreeGpu()


@pytest.mark.parametrize("kind", ["int32", "int16", "f16plain", "f16frame", "swar16", "unit", "pair", "k2_nowait",
                                  "k3_int32", "k3_nostrips", "k1_merge"])
@pytest.mark.parametrize("ds,var,opts", [("syn_small", "default", []), ("syn_short", "default", []),
                                         ("syn_small", "r64_pam250", ["-r", "64", "-M", cases.PAM250, "-y", "2"])])
def test_forced_score_encoding_matches_golden(kind, ds, var, opts, dataset, golden, tmp_path):
    """Every K2 encoding stays covered: the f16 kernel runs by default when all
    scores fit f16's exact-integer range, the int16 one above that, int32 when
    scores may exceed int16. Forced with GHOSTM_K2 each reproduces the golden."""
    d = dataset(ds)
    env = ({"GHOSTM_K3": "int32"} if kind == "k3_int32" else
           {"GHOSTM_K3_STRIPS": "0"} if kind == "k3_nostrips" else
           {"GHOSTM_K1": "merge"} if kind == "k1_merge" else
           {"GHOSTM_K2_NOWAIT": "1"} if kind == "k2_nowait" else {"GHOSTM_K2": kind})
    text, st = _gpu_text(d, opts, env, str(tmp_path / "g.out"))
    (tmp_path / "g.out").write_bytes(text)
    assert cases.sha256(str(tmp_path / "g.out")) == golden["aln"][f"{ds}/{var}"]["sha256"]
    assert st["traceback_launches"] > 0
    if kind == "k3_int32":
        assert st["traceback_launches_key"] == 0
    elif kind == "k3_nostrips":  # every hit's key DP on all of its group's strips
        assert st["traceback_launches_strips"] == 0 and st["traceback_launches_key"] > 0
    elif kind == "k1_merge":
        assert st["seed_runs_hash"] == 0
    elif kind == "k2_nowait":  # K2 launches without a host wait, timings resolved at the end
        assert st["score_launches_framed"] == st["score_launches"] > 0 and st["score_cells"] > 0
    elif kind == "f16plain":
        assert st["score_launches_half"] == st["score_launches"] > 0 and st["score_launches_framed"] == 0
    elif kind == "f16frame":  # the f16-number frame (k_score16f<S, false>), guarded where needed
        assert st["score_launches_framed"] == st["score_launches"] > 0 and st["score_launches_swar"] == 0
    elif kind == "swar16":  # integer patterns with 16-bit profile rows (k_score16f<S, true>)
        assert st["score_launches_swar"] == st["score_launches"] > 0 and st["score_launches_unit"] == 0
    elif kind == "unit":  # ... with unit-pair profile words (k_score16f<S, true, true>), however sparse
        assert st["score_launches_unit"] == st["score_launches"] > 0
    elif kind == "pair":  # the pair-table kernel (k_score_pair), however dense
        assert st["score_launches_pair"] == st["score_launches"] > 0
    else:
        assert st["score_launches"] > 0 and st["score_launches_half"] == 0
        assert st["score_launches_packed"] == (st["score_launches"] if kind == "int16" else 0)


def test_default_encoding_is_f16_when_scores_fit(dataset, golden, tmp_path):
    d = dataset("syn_small")
    text, st = _gpu_text(d, [], {}, str(tmp_path / "g.out"))
    assert st["score_launches_half"] == st["score_launches"] > 0
    assert st["score_launches_framed"] == st["score_launches"]  # k_score16f, the column-framed kernel
    assert st["score_launches_swar"] == st["score_launches"]  # ... over 16-bit integer patterns
    assert st["traceback_launches_key"] == st["traceback_launches"] > 0
    assert st["traceback_launches_strips"] == st["traceback_launches"]  # key DP by strip class
    assert st["seed_runs_hash"] > 0
    # PAM250 at L = 127 can reach 2159 > 2047: f16 runs with the re-score guard
    text2, st2 = _gpu_text(d, ["-M", cases.PAM250, "-G", "8", "-E", "1", "-y", "2"], {},
                            str(tmp_path / "p.out"))
    assert st2["score_launches_half"] == st2["score_launches_packed"] == st2["score_launches"] > 0


@pytest.mark.parametrize("ds,var,opts", [("syn_small", "pam250_g8e1", ["-M", cases.PAM250, "-G", "8", "-E", "1", "-y", "2"]),
                                         ("syn_small", "default", []), ("syn_dna", "default", [])])
def test_guarded_f16_rescores_exactly(ds, var, opts, dataset, golden, tmp_path):
    """With the guard forced low, many candidates go through the int16 re-score
    path of the guarded f16 kernel; the output is still the golden one."""
    d = dataset(ds)
    text, st = _gpu_text(d, opts, {"GHOSTM_K2_GUARD": "25"}, str(tmp_path / "g.out"))
    (tmp_path / "g.out").write_bytes(text)
    assert cases.sha256(str(tmp_path / "g.out")) == golden["aln"][f"{ds}/{var}"]["sha256"]
    assert st["score_rechecks"] > 0 and st["score_launches_half"] == st["score_launches"]


REF_GPU_VARIANTS = [v for v in cases.VARIANTS
                    if f"{v[0]}/{v[1]}" in ("protein_testset/y0", "readme_kat/default", "syn_small/default",
                                            "syn_small/r64_pam250", "syn_dna/default", "syn_chunks/default",
                                            "syn_short/default")]


@pytest.mark.skipif(not os.path.exists(cases.REF_PLUGIN), reason="reference build (oracle/_ref) absent")
@pytest.mark.parametrize("ds,var,opts,env", REF_GPU_VARIANTS, ids=[f"{v[0]}/{v[1]}" for v in REF_GPU_VARIANTS])
def test_reference_driver_on_this_plugin(ds, var, opts, env, dataset, golden, tmp_path):
    """The drop-in itself: the reference's own aligner.cpp (oracle/_ref, compiled from
    the reference sources, ghostm_ref_plugin: linked against libghostm_hip.so) run with -D 0 drives
    this repo's HIP kernels through the reference plugin ABI (InitGpu ... SearchNextGpu,
    CalculateScoreGpu ... FreeGpu) and must print the reference CPU path's bytes."""
    d = dataset(ds)
    out = str(tmp_path / "ref_gpu.out")
    cases.run_aln(cases.REF_PLUGIN, d, list(opts) + ["-D", "0"], env, out)
    assert cases.sha256(out) == golden["aln"][f"{ds}/{var}"]["sha256"]


@pytest.mark.parametrize("ds,opts", [("syn_small", []), ("syn_dna", []), ("syn_chunks", [])])
def test_device_records_equal_host_records(ds, opts, dataset, tmp_path):
    """The device-resident hit records (the multi-GPU gather payload) are the
    host records byte for byte: built per segment on the device (device merge,
    syn_small / syn_dna) or uploaded from the host merge (syn_chunks)."""
    d = dataset(ds)
    with Session(["-i", f"{d}/q", "-d", f"{d}/db", "-o", str(tmp_path / "x"), "-D", "0"] + opts) as s:
        s.run()
        host = s.hits()
        dev = s.device_hits().cpu().numpy()
        s.run()  # records are rebuilt per run, not appended
        dev2 = s.device_hits().cpu().numpy()
    assert len(host) > 0
    assert dev.tobytes() == host.tobytes()
    assert dev2.tobytes() == host.tobytes()


def test_wide_band_traceback_uses_key_kernel(dataset, golden, tmp_path):
    """-r 64 (cfg 5 style: PAM250, traceback window L + 2e*2*64 = 639 columns)
    runs the 17-bit-ml key traceback and still reproduces the golden output."""
    d = dataset("syn_small")
    opts = ["-r", "64", "-M", cases.PAM250, "-y", "2"]
    text, st = _gpu_text(d, opts, {}, str(tmp_path / "g.out"))
    (tmp_path / "g.out").write_bytes(text)
    assert cases.sha256(str(tmp_path / "g.out")) == golden["aln"]["syn_small/r64_pam250"]["sha256"]
    assert st["traceback_launches_key"] == st["traceback_launches"] > 0


@pytest.mark.parametrize("mode", ["default", "priv", "f16frame", "f16plain", "int16", "0", "keyframe0"])
@pytest.mark.parametrize("ds,var,opts", [("syn_small", "default", []), ("syn_dna", "default", []),
                                         ("syn_chunks", "default", []), ("protein_testset", "y2", ["-y", "2"]),
                                         ("syn_small", "r64_pam250", ["-r", "64", "-M", cases.PAM250, "-y", "2"])])
def test_traceback_scan_modes_match_golden(mode, ds, var, opts, dataset, golden, tmp_path):
    """Two-pass traceback (K3a scores-only scan, then the key DP over columns
    0..j* in j*-sorted order) in its encodings (default: the column-framed scan
    over 16-bit integer patterns; priv: the same scan reading a bank-private
    unit-word table; f16frame, f16plain, int16), and the single-pass traceback
    (GHOSTM_K3_SCAN=0): each reproduces the golden output. After a scan the key
    DP runs with its column-framed E chain (k_traceback_key FRAME);
    keyframe0 (GHOSTM_K3_KEYFRAME=0) keeps the unframed one."""
    d = dataset(ds)
    env = ({} if mode == "default" else {"GHOSTM_K3_KEYFRAME": "0"} if mode == "keyframe0"
           else {"GHOSTM_K3_SCAN": mode})
    text, st = _gpu_text(d, opts, env, str(tmp_path / "g.out"))
    (tmp_path / "g.out").write_bytes(text)
    assert cases.sha256(str(tmp_path / "g.out")) == golden["aln"][f"{ds}/{var}"]["sha256"]
    assert st["traceback_launches"] > 0
    assert st["traceback_launches_keyframe"] == (0 if mode in ("0", "keyframe0") else st["traceback_launches"])
    if mode == "0":
        assert st["traceback_launches_scan"] == 0 and st["traceback_scan_cells"] == 0
    else:
        # default: the framed scan over 16-bit integer patterns; the others not
        swar = mode in ("default", "priv", "keyframe0")
        assert st["traceback_launches_scan_swar"] == (st["traceback_launches"] if swar else 0)
        assert st["traceback_launches_scan"] == st["traceback_launches"]
        assert st["traceback_scan_cells"] > 0
        # the key DP runs only columns 0..j*: fewer cells than the scan covered
        assert st["traceback_cells"] < st["traceback_scan_cells"]


@pytest.mark.parametrize("mode", ["thread", "wave", "wave_cap40"])
@pytest.mark.parametrize("ds,var,opts", [("syn_small", "default", []), ("syn_small", "b3", ["-b", "3"]),
                                         ("syn_small", "b20_t1", ["-b", "20", "-t", "1", "-y", "2"]),
                                         ("syn_dna", "b5_y2", ["-b", "5", "-y", "2"]),
                                         ("protein_testset", "y2", ["-y", "2"]),
                                         ("syn_short", "default", [])])
def test_merge_modes_match_golden(mode, ds, var, opts, dataset, golden, tmp_path):
    """K4 with one thread per name group (k_merge) and with one wave per group
    (k_merge_wave: wave-parallel partitions of std::sort's introsort in LDS);
    wave_cap40 sends every group above 40 keys to the wave kernel's one-lane
    fallback, so both branches run in one launch. Each reproduces the golden."""
    d = dataset(ds)
    env = {"GHOSTM_K4": "thread"} if mode == "thread" else {"GHOSTM_K4": "wave"}
    if mode == "wave_cap40":
        env["GHOSTM_K4_CAP"] = "40"
    text, st = _gpu_text(d, opts, env, str(tmp_path / "g.out"))
    (tmp_path / "g.out").write_bytes(text)
    assert cases.sha256(str(tmp_path / "g.out")) == golden["aln"][f"{ds}/{var}"]["sha256"]
    assert st["merge_launches"] > 0
    assert st["merge_launches_wave"] == (0 if mode == "thread" else st["merge_launches"])


def test_gpu_ungapped_karlin_evalues(dataset, tmp_path):
    """§8 f4: PAM250 with -y 0 is outside the reference's gapped table and raises
    there (statistics.cpp:143-145); GHOSTM_KARLIN=ungapped prices it with the
    matrix's ungapped ideal parameters (bit-pinned in test_karlin.py). The bits
    column must be ((float)s * lambda - logf(K)) / (float)log(2) of the score -y 1
    prints for the same hit (statistics.cpp:40-44)."""
    from ghostm_amd import statistics
    d = dataset("syn_small")
    opts = ["-M", cases.PAM250]
    with pytest.raises(Exception):
        _gpu_text(d, opts + ["-y", "0"], {}, str(tmp_path / "a.out"))
    t0, _ = _gpu_text(d, opts + ["-y", "0"], {"GHOSTM_KARLIN": "ungapped"}, str(tmp_path / "b.out"))
    t1, _ = _gpu_text(d, opts + ["-y", "1"], {}, str(tmp_path / "c.out"))
    l0, l1 = t0.decode().splitlines(), t1.decode().splitlines()
    assert len(l0) == len(l1) > 0
    p = statistics.ungapped_ideal_karlin(cases.PAM250)
    lam, logk, ln2 = np.float32(p.lambda_), np.log(np.float32(p.K)), np.float32(np.log(2.0))
    for a, b in zip(l0, l1):
        fa, fb = a.split("\t"), b.split("\t")
        assert fa[:2] == fb[:2]
        want = (np.float32(int(fb[2])) * lam - logk) / ln2
        assert float(fa[8]) == pytest.approx(float(want), rel=1e-5)  # %g keeps 6 digits
        assert float(fa[7]) >= 0.0  # underflows to 0 for long exact matches, as in float


def test_stats_sized_writes_only_the_callers_fields(dataset, tmp_path):
    """GhostmSessionStatsSized: a caller built against an older, shorter
    GhostmStats gets exactly its prefix; the return value is the library's size."""
    d = dataset("syn_small")
    lib = native.load()
    with Session(["-i", f"{d}/q", "-d", f"{d}/db", "-o", str(tmp_path / "x"), "-D", "0"]) as s:
        s.run()
        full = native.GhostmStats()
        assert lib.GhostmSessionStatsSized(s._h, ctypes.byref(full), ctypes.sizeof(full)) == ctypes.sizeof(full)
        buf = (ctypes.c_ubyte * ctypes.sizeof(full))()
        assert lib.GhostmSessionStatsSized(s._h, ctypes.cast(buf, ctypes.POINTER(native.GhostmStats)), 64) \
            == ctypes.sizeof(full)
        raw = bytes(buf)
        assert raw[:64] == bytes(full)[:64] and not any(raw[64:])
        assert full.candidates > 0 and s.stats()["candidates"] == full.candidates
