import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import cases  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def built():
    """The native library, CLI and oracle binaries (built once if missing)."""
    need = [cases.GHOSTM, cases.ORACLE, os.path.join(REPO, "ghostm_amd", "lib", "libghostm_hip.so")]
    if not all(os.path.exists(p) for p in need):
        subprocess.run(["make", "-C", os.path.join(REPO, "ghostm_amd", "csrc"), "-j8"], check=True)
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "all"], check=True)
    return True


_HASH_CHECKED = {}


def library_hash_mismatch() -> str | None:
    """None when ghostm_amd/lib's product libraries were built from this tree's
    sources (GhostmBuildInfo's "src <hash>" = ghostm_amd/srchash.py over csrc/ and
    the header), else what differs. Read in a child process, so this process
    never loads a library the tests did not ask for."""
    from ghostm_amd import srchash

    want = srchash.tree_hash()
    lib_dir = os.path.join(REPO, "ghostm_amd", "lib")
    probs = []
    for name in ("libghostm_hip.so", "libghostm_hip_poison.so"):
        path = os.path.join(lib_dir, name)
        if not os.path.exists(path):
            probs.append(f"{name} missing")
            continue
        code = ("import ctypes, sys; l = ctypes.CDLL(sys.argv[1]); l.GhostmBuildInfo.restype = ctypes.c_char_p; "
                "print(l.GhostmBuildInfo().decode())")
        r = subprocess.run([sys.executable, "-c", code, path], capture_output=True, text=True)
        got = srchash.info_hash(r.stdout)
        if got != want:
            probs.append(f"{name}: src {got} (tree {want})")
    stray = sorted(n for n in os.listdir(lib_dir) if n.endswith(".so")
                   and n not in ("libghostm_hip.so", "libghostm_hip_poison.so"))
    if stray:
        probs.append(f"A/B builds in ghostm_amd/lib: {stray} (tools/altlib.sh writes ab_libs/)")
    return "; ".join(probs) or None


@pytest.fixture(autouse=True)
def _library_built_from_tree(request):
    """Every GPU test runs only on libraries built from the sources in this tree
    (a pushed .so older than csrc/ would test other code)."""
    if request.node.get_closest_marker("gpu") is None or os.environ.get("GHOSTM_LIB_PATH"):
        return
    if "r" not in _HASH_CHECKED:
        _HASH_CHECKED["r"] = library_hash_mismatch()
    if _HASH_CHECKED["r"]:
        pytest.fail("native library not built from this tree: " + _HASH_CHECKED["r"])


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(cases.GOLDEN, "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def data_root(tmp_path_factory, built):
    return str(tmp_path_factory.mktemp("ghostm_data"))


@pytest.fixture(scope="session")
def dataset(data_root):
    def make(name):
        return cases.build_dataset(name, data_root)
    return make
