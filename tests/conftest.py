import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


@pytest.fixture(scope="session")
def corpus():
    return dict(np.load(os.path.join(GOLDEN, "ed25519_corpus.npz")))


@pytest.fixture(scope="session")
def merkle_cases():
    return dict(np.load(os.path.join(GOLDEN, "merkle_cases.npz")))


@pytest.fixture(scope="session")
def manifest():
    import json
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle_c():
    import cv_oracle
    cv_oracle.lib()
    return cv_oracle


@pytest.fixture(scope="session")
def host_harness():
    """The product's per-lane device code compiled for the CPU (tests/host_harness.cpp)."""
    import ctypes
    if os.environ.get("CV_HOST_LIB"):        # a prebuilt variant (tests/sanitize: ASan + UBSan build)
        return ctypes.CDLL(os.environ["CV_HOST_LIB"])
    lib = os.path.join(REPO, "tests", "_build", "libcvhost.so")
    src = os.path.join(REPO, "tests", "host_harness.cpp")
    deps = [src] + [os.path.join(REPO, "corda_amd", "csrc", f) for f in os.listdir(os.path.join(REPO, "corda_amd", "csrc"))
                    if f.endswith(".h")]
    if not os.path.exists(lib) or any(os.path.getmtime(d) > os.path.getmtime(lib) for d in deps):
        os.makedirs(os.path.dirname(lib), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", "-DCV_BOUNDS_CHECK", "-fPIC", "-shared", src,
                        "-o", lib], check=True)
    return ctypes.CDLL(lib)


@pytest.fixture(scope="session")
def engine():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from corda_amd import native
    e = native.Engine(0)
    yield e
    e.close()
