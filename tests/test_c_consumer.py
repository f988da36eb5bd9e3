"""The C-ABI from plain C (tests/c_consumer/cv_consumer.c): include/cordaverify.h compiles as C99 under
-pedantic -Werror, the program links against the in-tree library alone, and drives the drop-in entry points the way
a JNI / JNA / cgo binding would — no Python or torch between it and the engine.  CPU: the host-only
entry points and cv_open's CV_E_NO_DEVICE; GPU: the golden corpus' verdicts and status bytes through the
synchronous, bounded (_ex), asynchronous and pinned-input forms."""
import os
import subprocess

import numpy as np
import pytest

from corda_amd import native

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "c_consumer", "cv_consumer.c")


def _build(tmp_path) -> str:
    exe = str(tmp_path / "cv_consumer")
    lib = os.path.abspath(native.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror", "-O1",
                    "-I", os.path.join(REPO, "include"), SRC, lib, f"-Wl,-rpath,{os.path.dirname(lib)}", "-o", exe],
                   check=True)
    return exe


def _fixture(corpus, path) -> str:
    n = corpus["pk"].shape[0]
    with open(path, "wb") as f:
        f.write(b"CVF1")
        f.write(np.array([n, corpus["arena"].size], np.uint64).tobytes())
        for k, dt in (("pk", np.uint8), ("sig", np.uint8), ("off", np.uint64), ("len", np.uint32),
                      ("verdict", np.uint8), ("status", np.uint8), ("arena", np.uint8)):
            f.write(np.ascontiguousarray(corpus[k], dtype=dt).tobytes())
    return str(path)


def test_c_consumer_host_only(tmp_path, corpus):
    """Builds as C99; the host-only entry points answer without a device; without a GPU cv_open returns
    CV_E_NO_DEVICE (exit 3) instead of falling back to anything."""
    exe = _build(tmp_path)
    fx = _fixture(corpus, tmp_path / "corpus.cvf")
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")   # host-only, even on a GPU box
    r = subprocess.run([exe, fx], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 3, (r.returncode, r.stdout, r.stderr)
    assert "host-only checks: ok" in r.stdout, r.stdout + r.stderr


def test_c_consumer_rejects_bad_fixture(tmp_path):
    exe = _build(tmp_path)
    bad = tmp_path / "bad.cvf"
    bad.write_bytes(b"XXXX")
    r = subprocess.run([exe, str(bad)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "usage" in r.stderr


@pytest.mark.gpu
def test_c_consumer_golden_corpus_on_gpu(tmp_path, corpus):
    """Every corpus record's verdict bit and status byte through the C entry points, at 1, 64, 699 and 2,114
    records (ragged last bitmap words), the arena bound one byte short, two async calls waited out of order, and
    inputs in cv_host_alloc memory."""
    exe = _build(tmp_path)
    fx = _fixture(corpus, tmp_path / "corpus.cvf")
    r = subprocess.run([exe, fx], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "all checks passed" in r.stdout
