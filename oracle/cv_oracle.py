"""ctypes wrapper for oracle/_build/libcvoracle.so (the C restatement).

TEST INFRASTRUCTURE ONLY — used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# CV_ORACLE_LIB: a prebuilt variant of the same C file (tests/sanitize: ASan + UBSan build)
_LIB_PATH = os.environ.get("CV_ORACLE_LIB") or os.path.join(_HERE, "_build", "libcvoracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        l = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        l.cvo_verify.argtypes = [u8p, u8p, u8p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int)]
        l.cvo_verify.restype = ctypes.c_int
        l.cvo_verify_batch.argtypes = [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_int]
        l.cvo_verify_batch.restype = ctypes.c_int
        l.cvo_merkle_tx_ids.argtypes = [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        l.cvo_merkle_tx_ids.restype = ctypes.c_int
        l.cvo_sha256.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        l.cvo_sha512.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        l.cvo_abyte.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        l.cvo_abyte.restype = ctypes.c_int
        _lib = l
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def verify_one(pk: bytes, msg: bytes, sig: bytes):
    """Returns (status, accepted)."""
    ok = ctypes.c_int(0)
    mb = (ctypes.c_uint8 * max(1, len(msg))).from_buffer_copy(msg + b"\0")
    st = lib().cvo_verify((ctypes.c_uint8 * 32).from_buffer_copy(pk), (ctypes.c_uint8 * 64).from_buffer_copy(sig),
                          mb, len(msg), ctypes.byref(ok))
    return st, bool(ok.value)


def verify_batch(pk: np.ndarray, sig: np.ndarray, arena: np.ndarray, off: np.ndarray, ln: np.ndarray,
                 nthreads: int = 1):
    """pk (n,32) u8, sig (n,64) u8, arena u8, off u64, ln u32 -> (verdict u8[n], status u8[n])."""
    n = pk.shape[0]
    pk = np.ascontiguousarray(pk, np.uint8)
    sig = np.ascontiguousarray(sig, np.uint8)
    arena = np.ascontiguousarray(arena, np.uint8)
    if arena.size == 0:
        arena = np.zeros(1, np.uint8)
    off = np.ascontiguousarray(off, np.uint64)
    ln = np.ascontiguousarray(ln, np.uint32)
    verdict = np.zeros(n, np.uint8)
    status = np.zeros(n, np.uint8)
    lib().cvo_verify_batch(n, _ptr(pk), _ptr(sig), _ptr(arena), _ptr(off), _ptr(ln), _ptr(verdict),
                           _ptr(status), int(nthreads))
    return verdict, status


def merkle_tx_ids(arena: np.ndarray, leaf_off: np.ndarray, leaf_len: np.ndarray, tx_leaf_begin: np.ndarray):
    ntx = tx_leaf_begin.shape[0] - 1
    arena = np.ascontiguousarray(arena, np.uint8)
    if arena.size == 0:
        arena = np.zeros(1, np.uint8)
    leaf_off = np.ascontiguousarray(leaf_off, np.uint64)
    leaf_len = np.ascontiguousarray(leaf_len, np.uint32)
    tx_leaf_begin = np.ascontiguousarray(tx_leaf_begin, np.uint32)
    ids = np.zeros((ntx, 32), np.uint8)
    status = np.zeros(ntx, np.uint8)
    lib().cvo_merkle_tx_ids(ntx, _ptr(arena), _ptr(leaf_off), _ptr(leaf_len), _ptr(tx_leaf_begin), _ptr(ids),
                            _ptr(status))
    return ids, status


def sha256(b: bytes) -> bytes:
    out = (ctypes.c_uint8 * 32)()
    buf = (ctypes.c_uint8 * max(1, len(b))).from_buffer_copy(b + b"\0")
    lib().cvo_sha256(out, buf, len(b))
    return bytes(out)


def sha512(b: bytes) -> bytes:
    out = (ctypes.c_uint8 * 64)()
    buf = (ctypes.c_uint8 * max(1, len(b))).from_buffer_copy(b + b"\0")
    lib().cvo_sha512(out, buf, len(b))
    return bytes(out)


def abyte(pk: bytes):
    out = (ctypes.c_uint8 * 32)()
    st = lib().cvo_abyte((ctypes.c_uint8 * 32).from_buffer_copy(pk), out)
    return st, bytes(out)
