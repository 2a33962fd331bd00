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
