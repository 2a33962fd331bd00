"""GPU `qry` formatter (include/ghostm_hip.h GhostmFormatQueriesGpu,
replacing QueryCreator's coding and six-frame translation, query_creator.cpp:242-324,
388-423).

`ghostm qry -D 0` must write the same bytes as the CPU formatter, whose files are
pinned to the reference program by tests/test_formatter.py: every dataset's query
options, plus edge cases the reference handles (reads shorter / longer than the
chunk's first read, ambiguous and gap letters, lower case, stop/ATG runs, records
over the width, one-letter records, several chunks)."""
import os
import subprocess

import pytest

import cases

pytestmark = pytest.mark.gpu

PROTEIN_EDGE = """>over_width
MKTAYIAKQRQISFVKSHFSRQLEERLGLIEVQAPILSRVGDGTQDNLSGAEKAVQVKVKALPDAQFEVVHSLAKWKRQTLGQHDFSAGEGLYTHMKALRPDEDRLSPLHSVYVDQWDWERVMGDGERQFSTLKSTVEAIWAGIKATEAAVSEEFGLAPF
>lower
acdefghiklmnpqrstvwy
>ambig
BZJUOX*acdBZ
>one
W
>empty_line_between

MKV
>trailing_plus
MKVL+
"""

DNA_EDGE = """>r0 first read sets the length
ATGAAATAGCCCATGGGGTGATTTTAAATGCCCGGGTAGATGNNNACGT
>r1 shorter
ATGCCCTAA
>r2 longer than the first
ATGAAATAGCCCATGGGGTGATTTTAAATGCCCGGGTAGATGNNNACGTACGTACGTTTT
>r3 lower case and gaps
atgaaa-tagcccatgggRYtgattttaaatgcccgggtagatgnnnacgt
>r4 stops everywhere
TAATAGTGATAATAGTGATAATAGTGATAATAGTGATAATAGTGATAAT
>r5 empty

>r6 reverse strand ATG
CATCATCATTTATTATTACATCATCATTTATTATTACATCATCATTTAT
"""


def _qry_files(d, prefix):
    return sorted(f for f in os.listdir(d) if f.startswith(prefix + "_") or f == prefix + ".inf")


def _both(fa, tmp_path, opts):
    for dev, out in ((None, "cpu"), ("0", "gpu")):
        cmd = [cases.GHOSTM, "qry", "-i", str(fa), "-o", str(tmp_path / out)] + opts
        if dev is not None:
            cmd += ["-D", dev]
        r = subprocess.run(cmd, capture_output=True, check=True)
        yield r.stderr
    cpu = _qry_files(str(tmp_path), "cpu")
    gpu = _qry_files(str(tmp_path), "gpu")
    assert [f[3:] for f in cpu] == [f[3:] for f in gpu]
    for a, b in zip(cpu, gpu):
        assert (tmp_path / a).read_bytes() == (tmp_path / b).read_bytes(), a


@pytest.mark.parametrize("name", ["protein_testset", "readme_kat", "syn_small", "syn_dna", "syn_short",
                                  "syn_chunks"])
def test_qry_gpu_matches_cpu(name, dataset, tmp_path):
    """Every dataset's query files from `qry -D 0` equal the CPU formatter's (and so
    the reference's: test_formatter.py)."""
    d = dataset(name)
    _, args = [t for t in cases.DATASETS[name] if t[0] == "qry"][0]
    a = [x.format(d=d, golden=cases.GOLDEN) for x in args]
    a[a.index("-o") + 1] = str(tmp_path / "q")
    subprocess.run([cases.GHOSTM, "qry"] + a + ["-D", "0"], check=True, capture_output=True)
    want = _qry_files(d, "q")
    have = _qry_files(str(tmp_path), "q")
    assert want == have
    for f in want:
        assert cases.sha256(os.path.join(d, f)) == cases.sha256(os.path.join(str(tmp_path), f)), f


@pytest.mark.parametrize("opts", [[], ["-l", "20"], ["-l", "500"], ["-l", "127"]])
def test_qry_gpu_protein_edges(opts, tmp_path):
    fa = tmp_path / "p.fa"
    fa.write_text(PROTEIN_EDGE)
    err_cpu, err_gpu = list(_both(fa, tmp_path, opts))
    assert err_cpu.count(b"warning") == err_gpu.count(b"warning")


@pytest.mark.parametrize("opts", [["-t", "d"], ["-t", "d", "-l", "30"], ["-t", "d", "-l", "600"]])
def test_qry_gpu_dna_edges(opts, tmp_path):
    """Six frames with the first read's length, stop masking until ATG on both
    strands, N and gap letters, shorter/longer/empty reads."""
    fa = tmp_path / "d.fa"
    fa.write_text(DNA_EDGE)
    err_cpu, err_gpu = list(_both(fa, tmp_path, opts))
    assert err_cpu.count(b"warning") == err_gpu.count(b"warning")
