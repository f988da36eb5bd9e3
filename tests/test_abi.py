"""The drop-in boundary on CPU: the C-ABI library loads, exports every symbol include/*.h declares,
and fails loudly (no silent fallback) when there is no GPU."""
import os
import re

import numpy as np
import pytest
import torch

from corda_amd import native

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    names = set()
    for h in os.listdir(os.path.join(REPO, "include")):
        if h.endswith(".h"):
            src = open(os.path.join(REPO, "include", h)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            names |= set(re.findall(r"\b(cv_[a-z0-9_]+)\s*\(", src))
    return names


def test_library_exports_every_declared_symbol():
    lib = native.load()
    declared = _header_functions()
    assert len(declared) >= 14
    for name in declared:
        assert hasattr(lib, name), f"{name} declared in include/ but not exported"
    assert set(native.EXPORTED) == declared


def test_only_declared_symbols_exported():
    """the product library exports the header's cv_* entry points and nothing of its own
    beyond them (the cvk_* kernel launchers and test hooks have hidden visibility)."""
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", native.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    ours = {ln.split()[-1] for ln in out.splitlines() if ln.split() and ln.split()[1] in "TtDdBbRrWwVv"
            and ln.split()[-1].startswith(("cv", "_Z"))}
    assert {s for s in ours if s.startswith("cvk")} == set(), sorted(ours)
    assert {s for s in ours if s.startswith("cv_")} == _header_functions()


def test_msg_extent():
    lib = native.load()
    off = np.array([5, 100, 7], np.uint64)
    ln = np.array([10, 0, 300], np.uint32)
    assert lib.cv_msg_extent(3, native._p(off), native._p(ln)) == 307
    assert lib.cv_msg_extent(0, None, None) == 0
    big_off = np.arange(3 << 20, dtype=np.uint64) * 3
    assert lib.cv_msg_extent(big_off.size, native._p(big_off), native._p(np.full(big_off.size, 3, np.uint32))) == 9 << 20


def test_version_and_strerror():
    lib = native.load()
    assert b"gfx950" in lib.cv_version()
    assert lib.cv_strerror(0) == b"ok"
    assert lib.cv_strerror(-1).startswith(b"no HIP device")


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure mode")
def test_no_gpu_fails_loudly():
    with pytest.raises(native.NativeUnavailable):
        native.Engine(0)
    with pytest.raises(native.NativeUnavailable):      # and the process-wide engine neither hangs nor falls back
        native.default_engine()


def test_null_context_rejected():
    lib = native.load()
    assert lib.cv_ed25519_verify_batch(None, 1, None, None, None, None, None, None, None) == -3
    assert lib.cv_merkle_tx_ids(None, 1, None, None, None, None, None) == -3
    assert lib.cv_close(None) is None


def test_tx_verdicts_host_only():
    bm = np.array([0b1011], np.uint64)
    assert native.tx_verdicts(bm, np.array([0, 2, 4, 4], np.uint32)).tolist() == [1, 0, 0]


def test_bitmap_to_bools():
    bm = np.array([1 | (1 << 63), 2], np.uint64)
    b = native.bitmap_to_bools(bm, 66)
    assert b[0] and b[63] and b[65] and not b[64] and b.sum() == 3


def test_dedupe_maps_repeated_keys():
    """Host key dedupe (the auto-keyed decision of cv_ed25519_verify_batch): every signature maps to
    the distinct key with its bytes, first-seen order."""
    rng = np.random.default_rng(7)
    keys = rng.integers(0, 256, (100, 32), dtype=np.uint8)
    order = rng.integers(0, 100, 1000)
    order[:100] = np.arange(100)                           # every key appears, first in index order
    pk = keys[order]
    idx, nk = native.dedupe_keys(pk)
    assert nk == 100
    assert np.array_equal(idx, order)
    assert native.dedupe_keys(rng.integers(0, 256, (1000, 32), dtype=np.uint8)) is None   # all distinct


def test_dedupe_resists_shared_key_bytes():
    """keys are untrusted, so a batch whose keys agree on bytes 8..15 (the old hash input)
    must not collapse into one probe chain.  2^15 distinct keys x 8 signatures (the keyed path's
    threshold), all sharing bytes 0..23 and differing only in the last 8: the seeded all-bytes hash
    keeps the dedupe of the 2^18 signatures linear."""
    import time
    n_keys = 1 << 15
    base = np.full(32, 0xA5, np.uint8)
    keys = np.tile(base, (n_keys, 1))
    keys[:, 24:32] = np.arange(n_keys, dtype=np.uint64).view(np.uint8).reshape(n_keys, 8)
    pk = np.repeat(keys, 8, axis=0)                       # each key signs 8 times, back to back
    t = time.perf_counter()
    idx, nk = native.dedupe_keys(pk)
    dt = time.perf_counter() - t
    assert nk == n_keys and np.array_equal(idx, np.repeat(np.arange(n_keys), 8))
    assert dt < 2.0, f"dedupe of 2^18 adversarial keys took {dt:.2f} s"


def test_dedupe_gate_and_threshold():
    """The keyed decision (cv_diag_dedupe_keys = the host dedupe cv_ed25519_verify_batch runs): above 4,096 signatures a
    birthday count over 4 sqrt(n) (512 .. 4,096) pseudo-random positions skips batches estimated below four
    signatures per key (a performance guess: the verdicts are the same either way).
    The full dedupe then takes the keyed path at eight or more signatures per distinct key, whatever the
    order of the records (a distinct-looking prefix included)."""
    rng = np.random.default_rng(9)
    keys = rng.integers(0, 256, (300, 32), dtype=np.uint8)
    pk = np.concatenate([keys] * 8)                          # 2400 sigs, 8 per key, prefix distinct
    idx, nk = native.dedupe_keys(pk)
    assert nk == 300 and np.array_equal(idx, np.tile(np.arange(300), 8))
    assert native.dedupe_keys(np.repeat(keys, 7, axis=0)) is None   # 7 per key: plain path
    # 2^20 signatures over a 1,024-key pool (the SURVEY §8(d) C2 variant), in random order
    pool = rng.integers(0, 256, (1024, 32), dtype=np.uint8)
    order = rng.integers(0, 1024, 1 << 20)
    idx, nk = native.dedupe_keys(pool[order])
    first = np.unique(order, return_index=True)[1]
    assert nk == 1024 and np.array_equal(pool[order][first[np.argsort(first)]][idx], pool[order])
    # 2^20 distinct keys: the gate declines without the full dedupe
    import time
    big = rng.integers(0, 256, (1 << 20, 32), dtype=np.uint8)
    t = time.perf_counter()
    assert native.dedupe_keys(big) is None
    assert time.perf_counter() - t < 0.5


def test_ids_output_checked():
    """the ids= output of the Merkle / transaction calls is checked before the library writes
    ntx * 32 bytes into it (no GPU needed: the check runs before any call)."""
    ok = np.zeros((4, 32), np.uint8)
    assert native._ids_out(ok, 4) is ok
    assert native._ids_out(None, 3).shape == (3, 32)
    for bad in (np.zeros((3, 32), np.uint8), np.zeros((4, 32), np.int8), np.zeros(128, np.uint8),
                np.zeros((4, 64), np.uint8)[:, ::2], np.zeros((8, 32), np.uint8)[::2]):
        with pytest.raises(ValueError):
            native._ids_out(bad, 4)
    ro = np.zeros((4, 32), np.uint8)
    ro.flags.writeable = False
    with pytest.raises(ValueError):
        native._ids_out(ro, 4)
