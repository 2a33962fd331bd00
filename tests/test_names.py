"""Sequence-name tables (ghostm_amd/csrc/formats.cpp NameTable, ReadNameLines),
compiled with g++ and compared with the reference's getline reading of .nam
files (query_reader.cpp): complete, short and unterminated files, empty names,
a missing file, slices and names added after a slice."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_name_tables_equal_getline(tmp_path):
    exe = str(tmp_path / "test_names")
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(HERE, "native", "test_names.cpp"),
                    os.path.join(os.path.dirname(HERE), "ghostm_amd", "csrc", "formats.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout
