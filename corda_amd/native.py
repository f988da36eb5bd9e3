"""ctypes binding of the C-ABI in include/cordaverify.h (corda_amd/libcordaverify.so).

This is the product path: there is no CPU fallback.  If the library is missing or no GPU is
present, the calls raise `NativeUnavailable` — loudly — instead of computing anything elsewhere.
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref
from typing import Optional, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# CV_LIB_PATH: load an alternative build of the same ABI (A/B tooling)
LIB_PATH = os.environ.get("CV_LIB_PATH") or os.path.join(HERE, "libcordaverify.so")

CV_OK = 0
CV_SIG_OK = 0
CV_SIG_BAD_KEY = 1
CV_TX_OK = 0
CV_TX_EMPTY = 1

# every symbol include/cordaverify.h declares (tests check the library exports all of them)
EXPORTED = (
    "cv_open", "cv_close", "cv_strerror", "cv_version", "cv_device_count",
    "cv_ed25519_verify_batch", "cv_merkle_tx_ids", "cv_merkle_tx_ids_ex", "cv_ed25519_sign_batch",
    "cv_tx_verdicts", "cv_ed25519_verify_device", "cv_ed25519_verify_device_timed", "cv_ed25519_sign_device", "cv_merkle_tx_ids_device",
    "cv_synchronize", "cv_calibrate", "cv_ed25519_verify_batch_keyed", "cv_key_cache_reserve", "cv_key_cache_stats",
    "cv_ed25519_verify_device_keyed", "cv_partial_merkle_verify", "cv_calibrate_cycles",
    "cv_diag_dedupe_keys", "cv_host_alloc", "cv_host_free", "cv_ed25519_verify_batch_async", "cv_wait",
    "cv_merkle_tx_ids_async", "cv_set_option", "cv_get_option", "cv_diag_stats",
    "cv_verify_transactions", "cv_verify_transactions_async", "cv_open_ex", "cv_msg_extent",
    "cv_ed25519_verify_batch_ex", "cv_merkle_tx_ids_bounded", "cv_verify_transactions_ex",
)

# cv_set_option names (include/cordaverify.h CV_OPT_*)
OPTIONS = {"tri_max": 1, "quad_max": 2, "drain_split": 3, "drain_split_pct": 4, "pipe_min": 5, "pipe_first": 6,
           "pipe_chunk": 7, "async_chunk": 8, "host_threads": 9, "small_zero_copy": 10, "small_direct_min": 11,
           "auto_keyed": 12, "shard_min": 13, "spread_min": 14, "merkle_chunk": 15,
           "prep_overlap_min": 16, "timeline": 17, "pipe_split": 18,
           "pipe_overlap_first": 19, "mid_pieces": 20,
           "pipe_slots": 21, "txs_merkle_stream": 22}
STATS = {"pipe": (0, ("plan_s", "pack_s", "wait_s", "enqueue_s", "sync_s", "calls", "subchunks", "direct_subchunks")),
         "small": (1, ("setup_s", "pack_s", "launch_s", "sync_s", "assemble_s", "calls")),
         "route": (2, ("calls", "routed_whole", "split_calls", "shards", "keyed_shards", "keyed_subchunks",
                       "merkle_calls", "merkle_subchunks")),
         "timeline": (3, ("ramp_ms", "dma_end_ms", "span_ms", "busy_ms", "idle_ms", "tail_ms", "result_copy_ms",
                          "first_subchunk", "merkle_busy_ms", "verify_busy_ms", "merkle_dma_end_ms", "groups",
                          "host_pre_ms", "host_post_ms", "calls"))}


class NativeUnavailable(RuntimeError):
    pass


class CvError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what}: {_lib.cv_strerror(code).decode() if _lib else code} (code {code})")
        self.code = code


_lib = None
_lock = threading.Lock()

_vp = ctypes.c_void_p
_sz = ctypes.c_size_t


def load():
    """Load the shared library (does not touch the GPU)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeUnavailable(f"{LIB_PATH} is missing: build it with `python -m corda_amd.build`")
        lib = ctypes.CDLL(LIB_PATH)
        lib.cv_open.argtypes = [ctypes.c_uint32, ctypes.POINTER(_vp)]
        lib.cv_open.restype = ctypes.c_int
        lib.cv_close.argtypes = [_vp]
        lib.cv_close.restype = None
        lib.cv_strerror.argtypes = [ctypes.c_int]
        lib.cv_strerror.restype = ctypes.c_char_p
        lib.cv_version.argtypes = []
        lib.cv_version.restype = ctypes.c_char_p
        lib.cv_device_count.argtypes = [_vp]
        lib.cv_device_count.restype = ctypes.c_int
        lib.cv_ed25519_verify_batch.argtypes = [_vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
        lib.cv_ed25519_verify_batch.restype = ctypes.c_int
        lib.cv_merkle_tx_ids.argtypes = [_vp, _sz, _vp, _vp, _vp, _vp, _vp]
        lib.cv_merkle_tx_ids.restype = ctypes.c_int
        lib.cv_merkle_tx_ids_ex.argtypes = [_vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp]
        lib.cv_merkle_tx_ids_async.argtypes = [_vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.POINTER(ctypes.c_uint64)]
        lib.cv_merkle_tx_ids_async.restype = ctypes.c_int
        lib.cv_verify_transactions.argtypes = [_vp, _sz] + [_vp] * 11
        lib.cv_verify_transactions.restype = ctypes.c_int
        lib.cv_verify_transactions_async.argtypes = [_vp, _sz] + [_vp] * 11 + [ctypes.POINTER(ctypes.c_uint64)]
        lib.cv_verify_transactions_ex.argtypes = [_vp, _sz, _vp, ctypes.c_uint64] + [_vp] * 10 + \
            [ctypes.POINTER(ctypes.c_uint64)]
        lib.cv_verify_transactions_ex.restype = ctypes.c_int
        lib.cv_merkle_tx_ids_bounded.argtypes = [_vp, _sz, _vp, ctypes.c_uint64] + [_vp] * 5 + \
            [ctypes.POINTER(ctypes.c_uint64)]
        lib.cv_merkle_tx_ids_bounded.restype = ctypes.c_int
        lib.cv_verify_transactions_async.restype = ctypes.c_int
        lib.cv_set_option.argtypes = [_vp, ctypes.c_int, ctypes.c_int64]
        lib.cv_set_option.restype = ctypes.c_int
        lib.cv_get_option.argtypes = [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]
        lib.cv_get_option.restype = ctypes.c_int
        lib.cv_diag_stats.argtypes = [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_double), _sz, ctypes.c_int]
        lib.cv_diag_stats.restype = ctypes.c_int
        lib.cv_open_ex.argtypes = [ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(_vp)]
        lib.cv_open_ex.restype = ctypes.c_int
        lib.cv_partial_merkle_verify.argtypes = [_vp, _sz, _sz, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp, _vp, _vp, _vp]
        lib.cv_partial_merkle_verify.restype = ctypes.c_int
        lib.cv_merkle_tx_ids_ex.restype = ctypes.c_int
        lib.cv_ed25519_sign_batch.argtypes = [_vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp]
        lib.cv_ed25519_sign_batch.restype = ctypes.c_int
        lib.cv_ed25519_verify_batch_async.argtypes = [_vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                                      ctypes.POINTER(ctypes.c_uint64)]
        lib.cv_ed25519_verify_batch_async.restype = ctypes.c_int
        lib.cv_ed25519_verify_batch_ex.argtypes = [_vp, _sz, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, _vp, _vp,
                                                   ctypes.POINTER(ctypes.c_uint64)]
        lib.cv_ed25519_verify_batch_ex.restype = ctypes.c_int
        lib.cv_wait.argtypes = [_vp, ctypes.c_uint64]
        lib.cv_wait.restype = ctypes.c_int
        lib.cv_host_alloc.argtypes = [_vp, _sz, ctypes.POINTER(_vp)]
        lib.cv_host_alloc.restype = ctypes.c_int
        lib.cv_host_free.argtypes = [_vp, _vp]
        lib.cv_host_free.restype = None
        lib.cv_msg_extent.argtypes = [_sz, _vp, _vp]
        lib.cv_msg_extent.restype = ctypes.c_uint64
        lib.cv_tx_verdicts.argtypes = [_sz, _vp, _vp, _vp]
        lib.cv_tx_verdicts.restype = ctypes.c_int
        lib.cv_ed25519_verify_device.argtypes = [_vp, ctypes.c_int, _sz, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
        lib.cv_ed25519_verify_device.restype = ctypes.c_int
        lib.cv_ed25519_verify_device_timed.argtypes = [_vp, ctypes.c_int, _sz, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                                       ctypes.POINTER(ctypes.c_float)]
        lib.cv_ed25519_verify_device_timed.restype = ctypes.c_int
        lib.cv_ed25519_sign_device.argtypes = [_vp, ctypes.c_int, _sz, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
        lib.cv_ed25519_sign_device.restype = ctypes.c_int
        lib.cv_merkle_tx_ids_device.argtypes = [_vp, ctypes.c_int, _sz, _sz, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
        lib.cv_merkle_tx_ids_device.restype = ctypes.c_int
        lib.cv_synchronize.argtypes = [_vp, ctypes.c_int]
        lib.cv_synchronize.restype = ctypes.c_int
        lib.cv_ed25519_verify_batch_keyed.argtypes = [_vp, _sz, _sz, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
        lib.cv_ed25519_verify_batch_keyed.restype = ctypes.c_int
        lib.cv_key_cache_reserve.argtypes = [_vp, _sz]
        lib.cv_key_cache_reserve.restype = ctypes.c_int
        lib.cv_key_cache_stats.argtypes = [_vp, ctypes.c_int, _vp]
        lib.cv_key_cache_stats.restype = ctypes.c_int
        lib.cv_ed25519_verify_device_keyed.argtypes = [_vp, ctypes.c_int, _sz, _sz, _vp, _vp, _vp, _vp, _vp, _vp,
                                                       _vp, _vp, _vp, ctypes.POINTER(ctypes.c_float)]
        lib.cv_ed25519_verify_device_keyed.restype = ctypes.c_int
        lib.cv_calibrate.argtypes = [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        lib.cv_calibrate.restype = ctypes.c_int
        lib.cv_calibrate_cycles.argtypes = [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        lib.cv_calibrate_cycles.restype = ctypes.c_int
        lib.cv_diag_dedupe_keys.argtypes = [_sz, _vp, _vp, ctypes.POINTER(_sz)]
        lib.cv_diag_dedupe_keys.restype = ctypes.c_int
        _lib = lib
        return lib


_C0 = ctypes.c_char * 0


def _p(a: Optional[np.ndarray]):
    """The array's data pointer as an int (c_void_p arguments).  Through the buffer protocol: ~0.4 us per
    pointer against ~3 us for ndarray.ctypes.data_as, which a notary-sized call pays seven times; arrays the
    buffer protocol refuses (read-only, non-contiguous) take the ctypes attribute."""
    if a is None:
        return None
    try:
        return ctypes.addressof(_C0.from_buffer(a))
    except (TypeError, ValueError, BufferError):
        return a.ctypes.data


def _u8(a, shape_last=None) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return a


def _msg_end(lib, off: np.ndarray, ln: np.ndarray) -> int:
    """max(off + len) — the arena bytes the records reach (multi-threaded in the library for big n)."""
    return int(lib.cv_msg_extent(off.shape[0], _p(off), _p(ln)))


def _ids_out(ids, ntx: int) -> np.ndarray:
    """The caller's optional ids output (the library writes ntx * 32 bytes into it): a new array when None,
    else it must be a writable, C-contiguous uint8 array of shape (ntx, 32) — a short or strided buffer would
    be written past its end or into the wrong bytes."""
    if ids is None:
        return np.zeros((ntx, 32), np.uint8)
    if not isinstance(ids, np.ndarray) or ids.dtype != np.uint8 or ids.shape != (ntx, 32):
        raise ValueError(f"ids must be a uint8 array of shape ({ntx}, 32)")
    if not ids.flags.c_contiguous or not ids.flags.writeable:
        raise ValueError("ids must be C-contiguous and writable")
    return ids


def _check(rc: int, what: str):
    if rc != CV_OK:
        raise CvError(rc, what)


class Engine:
    """One context over a set of GPUs (bit d of device_mask = HIP device d; 0 = all).

    Host-buffer methods mirror the JVM drop-in (synchronous unless *_async); *_device methods take device
    pointers (ints, e.g. torch.Tensor.data_ptr()) and an optional hipStream_t (int), and return
    immediately.  The context is thread-safe: calls from several Python threads run concurrently (ctypes
    releases the GIL) and the engine routes them over its devices.
    virtual_devices (cv_open_ex): each GPU of the mask appears that many times in this context (independent
    device slots: the multi-device routing on a one-GPU box).
    """

    def __init__(self, device_mask: int = 0, virtual_devices: int = 1):
        lib = load()
        h = _vp()
        if virtual_devices != 1:
            rc = lib.cv_open_ex(ctypes.c_uint32(device_mask), int(virtual_devices), ctypes.byref(h))
        else:
            rc = lib.cv_open(ctypes.c_uint32(device_mask), ctypes.byref(h))
        if rc != CV_OK:
            raise NativeUnavailable(f"cv_open failed: {lib.cv_strerror(rc).decode()} (code {rc})")
        self._lib = lib
        self._h = h
        self.mu = threading.Lock()
        self._inflight = {}

    def close(self):
        if self._h:
            self._lib.cv_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def device_count(self) -> int:
        return self._lib.cv_device_count(self._h)

    # ------------------------------------------------------------ host-buffer API
    def host_empty(self, shape, dtype=np.uint8) -> np.ndarray:
        """An uninitialised numpy array in pinned host memory (cv_host_alloc), freed with its last view.
        Host-buffer calls whose five input arrays are all pinned skip the engine's packing copy."""
        shape = (shape,) if isinstance(shape, int) else tuple(shape)
        nbytes = max(1, int(np.prod(shape)) * np.dtype(dtype).itemsize)
        ptr = _vp()
        _check(self._lib.cv_host_alloc(self._h, nbytes, ctypes.byref(ptr)), "cv_host_alloc")
        buf = (ctypes.c_uint8 * nbytes).from_address(ptr.value)
        weakref.finalize(buf, self._lib.cv_host_free, None, ctypes.c_void_p(ptr.value))
        return np.frombuffer(buf, dtype=dtype, count=int(np.prod(shape))).reshape(shape)

    def host_copy(self, a) -> np.ndarray:
        """A pinned copy of array a (host_empty + copy)."""
        a = np.ascontiguousarray(a)
        out = self.host_empty(a.shape, a.dtype)
        out[...] = a
        return out

    def verify_batch(self, pk, sig, arena, off, ln, want_status: bool = True) -> Tuple[np.ndarray, Optional[np.ndarray]]:
        """pk (n,32) u8, sig (n,64) u8, arena u8, off u64[n], ln u32[n] -> (bitmap u64[ceil(n/64)], status u8[n])."""
        pk = _u8(pk)
        sig = _u8(sig)
        n = pk.shape[0]
        if pk.size != n * 32 or sig.size != n * 64:
            raise ValueError("pk must be (n,32) and sig (n,64)")
        arena = _u8(arena) if arena is not None and np.asarray(arena).size else np.zeros(16, np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        ln = np.ascontiguousarray(ln, dtype=np.uint32)
        if off.shape[0] != n or ln.shape[0] != n:
            raise ValueError("off/len must have n entries")
        bitmap = np.zeros((n + 63) // 64, np.uint64)
        status = np.zeros(n, np.uint8) if want_status else None
        # the arena bound is checked by the engine's own staging scan (cv_ed25519_verify_batch_ex)
        rc = self._lib.cv_ed25519_verify_batch_ex(self._h, n, _p(pk), _p(sig), _p(arena), arena.size, _p(off), _p(ln),
                                                  _p(bitmap), _p(status), None)
        if rc == -3 and n and _msg_end(self._lib, off, ln) > arena.size:
            raise ValueError("message range exceeds the arena")
        _check(rc, "cv_ed25519_verify_batch")
        return bitmap, status

    def verify_batch_async(self, pk, sig, arena, off, ln, want_status: bool = True) -> int:
        """cv_ed25519_verify_batch_async: enqueue and return a ticket; wait(ticket) -> (bitmap, status).
        The arrays are kept referenced here until the wait (the engine may DMA from them until then)."""
        pk = _u8(pk)
        sig = _u8(sig)
        n = pk.shape[0]
        if pk.size != n * 32 or sig.size != n * 64:
            raise ValueError("pk must be (n,32) and sig (n,64)")
        arena = _u8(arena) if arena is not None and np.asarray(arena).size else np.zeros(16, np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        ln = np.ascontiguousarray(ln, dtype=np.uint32)
        if off.shape[0] != n or ln.shape[0] != n:
            raise ValueError("off/len must have n entries")
        bitmap = np.zeros((n + 63) // 64, np.uint64)
        status = np.zeros(n, np.uint8) if want_status else None
        t = ctypes.c_uint64()
        rc = self._lib.cv_ed25519_verify_batch_ex(self._h, n, _p(pk), _p(sig), _p(arena), arena.size, _p(off), _p(ln),
                                                  _p(bitmap), _p(status), ctypes.byref(t))
        if rc == -3 and n and _msg_end(self._lib, off, ln) > arena.size:
            raise ValueError("message range exceeds the arena")
        _check(rc, "cv_ed25519_verify_batch_async")
        with self.mu:
            self._inflight[t.value] = (bitmap, status, (pk, sig, arena, off, ln))
        return t.value

    def wait(self, ticket: int):
        """cv_wait: the results of an async call — (bitmap, status) for a verify, (ids, status) for Merkle ids."""
        with self.mu:
            a, b, keep = self._inflight.get(ticket, (None, None, None))
        _check(self._lib.cv_wait(self._h, ctypes.c_uint64(ticket)), "cv_wait")
        with self.mu:
            self._inflight.pop(ticket, None)
        del keep
        return a, b

    def verify_batch_keyed(self, keys, key_index, sig, arena, off, ln, want_status: bool = True):
        """keys (nk,32) distinct keys, key_index u32[n] -> (bitmap, status) exactly as verify_batch."""
        keys = _u8(keys)
        nk = keys.shape[0]
        key_index = np.ascontiguousarray(key_index, dtype=np.uint32)
        sig = _u8(sig)
        n = key_index.shape[0]
        if keys.size != nk * 32 or sig.size != n * 64:
            raise ValueError("keys must be (nk,32) and sig (n,64)")
        if n and int(key_index.max()) >= nk:
            raise ValueError("key_index out of range")
        arena = _u8(arena) if arena is not None and np.asarray(arena).size else np.zeros(16, np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        ln = np.ascontiguousarray(ln, dtype=np.uint32)
        if n and _msg_end(self._lib, off, ln) > arena.size:
            raise ValueError("message range exceeds the arena")
        bitmap = np.zeros((n + 63) // 64, np.uint64)
        status = np.zeros(n, np.uint8) if want_status else None
        _check(self._lib.cv_ed25519_verify_batch_keyed(self._h, n, nk, _p(keys), _p(key_index), _p(sig), _p(arena),
                                                       _p(off), _p(ln), _p(bitmap), _p(status)),
               "cv_ed25519_verify_batch_keyed")
        return bitmap, status

    def key_cache_reserve(self, max_keys: int):
        _check(self._lib.cv_key_cache_reserve(self._h, max_keys), "cv_key_cache_reserve")

    def key_cache_stats(self, device: int = 0) -> dict:
        out = np.zeros(4, np.uint64)
        _check(self._lib.cv_key_cache_stats(self._h, device, _p(out)), "cv_key_cache_stats")
        return {"resident": int(out[0]), "capacity": int(out[1]), "hits": int(out[2]), "misses": int(out[3])}

    def sign_batch(self, seeds, arena, off, ln) -> Tuple[np.ndarray, np.ndarray]:
        seeds = _u8(seeds)
        n = seeds.shape[0]
        arena = _u8(arena) if arena is not None and np.asarray(arena).size else np.zeros(16, np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        ln = np.ascontiguousarray(ln, dtype=np.uint32)
        pk = np.zeros((n, 32), np.uint8)
        sig = np.zeros((n, 64), np.uint8)
        _check(self._lib.cv_ed25519_sign_batch(self._h, n, _p(seeds), _p(arena), _p(off), _p(ln), _p(pk),
                                               _p(sig)), "cv_ed25519_sign_batch")
        return pk, sig

    @staticmethod
    def _merkle_args(arena, leaf_off, leaf_len, tx_leaf_begin, scan: bool = False):
        """The leaf arrays as the library takes them.  scan: also check the leaves against the arena here (the
        bounded entry points check it in the engine's own staging scan; this is their error path)."""
        tx_leaf_begin = np.ascontiguousarray(tx_leaf_begin, dtype=np.uint32)
        ntx = tx_leaf_begin.shape[0] - 1
        arena = _u8(arena) if arena is not None and np.asarray(arena).size else np.zeros(16, np.uint8)
        leaf_off = np.ascontiguousarray(leaf_off, dtype=np.uint64)
        leaf_len = np.ascontiguousarray(leaf_len, dtype=np.uint32)
        if leaf_off.size == 0:
            leaf_off = np.zeros(1, np.uint64)
            leaf_len = np.zeros(1, np.uint32)
        if leaf_off.shape[0] != leaf_len.shape[0] or (ntx > 0 and int(tx_leaf_begin[-1]) > leaf_off.shape[0]):
            raise ValueError("tx_leaf_begin reaches past the leaf arrays")
        if scan and ntx > 0 and int(tx_leaf_begin[-1]) and _msg_end(load(), leaf_off[:int(tx_leaf_begin[-1])],
                                                                    leaf_len[:int(tx_leaf_begin[-1])]) > arena.size:
            raise ValueError("leaf range exceeds the arena")
        return ntx, arena, leaf_off, leaf_len, tx_leaf_begin

    def _bounded_rc(self, rc: int, what: str, leaves):
        """A bounded call's return code: CV_E_ARGS from leaves past the arena (or wrapping) as ValueError, as
        the binding raised it when it scanned the leaves itself; any other error as CvError."""
        if rc == -3:
            self._merkle_args(*leaves, scan=True)   # raises ValueError for leaves past the arena
        _check(rc, what)

    def merkle_tx_ids(self, arena, leaf_off, leaf_len, tx_leaf_begin, ids=None) -> Tuple[np.ndarray, np.ndarray]:
        """WireTransaction.id of every transaction -> (ids (ntx,32) u8, status u8[ntx]).  ids: an optional
        output array (e.g. pinned, host_empty), so the ids are DMAed straight into it."""
        ntx, arena, leaf_off, leaf_len, tx_leaf_begin = self._merkle_args(arena, leaf_off, leaf_len, tx_leaf_begin)
        ids = _ids_out(ids, max(ntx, 0))
        st = np.zeros(max(ntx, 0), np.uint8)
        # the leaf-arena bound is checked by the engine's staging scan (cv_merkle_tx_ids_bounded)
        rc = self._lib.cv_merkle_tx_ids_bounded(self._h, ntx, _p(arena), arena.size, _p(leaf_off), _p(leaf_len),
                                                _p(tx_leaf_begin), _p(ids), _p(st), None)
        self._bounded_rc(rc, "cv_merkle_tx_ids_bounded", (arena, leaf_off, leaf_len, tx_leaf_begin))
        return ids, st

    def merkle_tx_ids_async(self, arena, leaf_off, leaf_len, tx_leaf_begin, ids=None) -> int:
        """cv_merkle_tx_ids_async: enqueue and return a ticket; wait(ticket) -> (ids, status)."""
        ntx, arena, leaf_off, leaf_len, tx_leaf_begin = self._merkle_args(arena, leaf_off, leaf_len, tx_leaf_begin)
        ids = _ids_out(ids, max(ntx, 0))
        st = np.zeros(max(ntx, 0), np.uint8)
        t = ctypes.c_uint64()
        rc = self._lib.cv_merkle_tx_ids_bounded(self._h, ntx, _p(arena), arena.size, _p(leaf_off), _p(leaf_len),
                                                _p(tx_leaf_begin), _p(ids), _p(st), ctypes.byref(t))
        self._bounded_rc(rc, "cv_merkle_tx_ids_bounded", (arena, leaf_off, leaf_len, tx_leaf_begin))
        with self.mu:
            self._inflight[t.value] = (ids, st, (arena, leaf_off, leaf_len, tx_leaf_begin))
        return t.value

    def _tx_args(self, arena, leaf_off, leaf_len, tx_leaf_begin, pk, sig, tx_sig_begin, ids, want_status,
                 want_sig_status):
        ntx, arena, leaf_off, leaf_len, tx_leaf_begin = self._merkle_args(arena, leaf_off, leaf_len, tx_leaf_begin)
        tx_sig_begin = np.ascontiguousarray(tx_sig_begin, dtype=np.uint32)
        if tx_sig_begin.shape[0] != ntx + 1:
            raise ValueError("tx_sig_begin must have ntx + 1 entries")
        pk = _u8(pk)
        sig = _u8(sig)
        nsig = int(tx_sig_begin[-1]) if ntx > 0 else 0
        if pk.size < nsig * 32 or sig.size < nsig * 64:
            raise ValueError("tx_sig_begin reaches past pk / sig")
        if pk.size == 0:
            pk, sig = np.zeros(32, np.uint8), np.zeros(64, np.uint8)
        ntx = max(ntx, 0)
        ids = _ids_out(ids, ntx)
        st = np.zeros(ntx, np.uint8) if want_status else None
        sst = np.zeros(nsig, np.uint8) if want_sig_status else None
        ok = np.zeros(ntx, np.uint8)
        args = (ntx, _p(arena), arena.size, _p(leaf_off), _p(leaf_len), _p(tx_leaf_begin), _p(pk), _p(sig),
                _p(tx_sig_begin), _p(ids), _p(st), _p(sst), _p(ok))
        return args, (ok, ids, st, sst), (arena, leaf_off, leaf_len, tx_leaf_begin, pk, sig, tx_sig_begin)

    def verify_transactions(self, arena, leaf_off, leaf_len, tx_leaf_begin, pk, sig, tx_sig_begin, ids=None,
                            want_status: bool = True, want_sig_status: bool = False):
        """cv_verify_transactions (SignedTransaction.verifySignatures' id + signature checks for a batch) ->
        (tx_ok u8[ntx], ids (ntx,32) u8, tx_status u8[ntx] or None, sig_status u8[nsig] or None)."""
        args, out, keep = self._tx_args(arena, leaf_off, leaf_len, tx_leaf_begin, pk, sig, tx_sig_begin, ids,
                                        want_status, want_sig_status)
        rc = self._lib.cv_verify_transactions_ex(self._h, *args, None)
        self._bounded_rc(rc, "cv_verify_transactions_ex", keep[:4])
        return out

    def verify_transactions_async(self, arena, leaf_off, leaf_len, tx_leaf_begin, pk, sig, tx_sig_begin, ids=None,
                                  want_status: bool = True, want_sig_status: bool = False) -> int:
        """cv_verify_transactions_async: enqueue and return a ticket; wait(ticket) -> (tx_ok, (ids, tx_status,
        sig_status))."""
        args, out, keep = self._tx_args(arena, leaf_off, leaf_len, tx_leaf_begin, pk, sig, tx_sig_begin, ids,
                                        want_status, want_sig_status)
        t = ctypes.c_uint64()
        rc = self._lib.cv_verify_transactions_ex(self._h, *args, ctypes.byref(t))
        self._bounded_rc(rc, "cv_verify_transactions_ex", keep[:4])
        with self.mu:
            self._inflight[t.value] = (out[0], out[1:], keep)
        return t.value

    # ------------------------------------------------------------ options and diagnostics
    def set_option(self, name: str, value: int):
        _check(self._lib.cv_set_option(self._h, OPTIONS[name], int(value)), f"cv_set_option({name})")

    def get_option(self, name: str) -> int:
        v = ctypes.c_int64()
        _check(self._lib.cv_get_option(self._h, OPTIONS[name], ctypes.byref(v)), f"cv_get_option({name})")
        return v.value

    def stats(self, kind: str, reset: bool = False) -> dict:
        which, names = STATS[kind]
        out = (ctypes.c_double * len(names))()
        rc = self._lib.cv_diag_stats(self._h, which, out, len(names), int(reset))
        if rc < 0:
            raise CvError(rc, "cv_diag_stats")
        return dict(zip(names, out))

    def partial_merkle_verify(self, kind, left, right, leaf_hash, tree_begin, root, check, check_begin
                              ) -> Tuple[np.ndarray, np.ndarray]:
        """Flat partial Merkle trees (include/cordaverify.h) -> (verdict[ntrees], status[ntrees])."""
        tree_begin = np.ascontiguousarray(tree_begin, dtype=np.uint32)
        check_begin = np.ascontiguousarray(check_begin, dtype=np.uint32)
        ntrees = tree_begin.shape[0] - 1
        nnodes = int(tree_begin[-1]) if ntrees > 0 else 0
        ncheck = int(check_begin[-1]) if ntrees > 0 else 0

        def pad(a, dt, shape):
            a = np.ascontiguousarray(a, dtype=dt)
            return a if a.size else np.zeros(shape, dt)
        kind = pad(kind, np.uint8, 1)
        left = pad(left, np.uint32, 1)
        right = pad(right, np.uint32, 1)
        leaf_hash = pad(leaf_hash, np.uint8, (1, 32))
        root = pad(root, np.uint8, (1, 32))
        check = pad(check, np.uint8, (1, 32))
        verdict = np.zeros(max(ntrees, 1), np.uint8)
        status = np.zeros(max(ntrees, 1), np.uint8)
        _check(self._lib.cv_partial_merkle_verify(self._h, ntrees, nnodes, _p(kind), _p(left), _p(right),
                                                  _p(leaf_hash), _p(tree_begin), _p(root), ncheck, _p(check),
                                                  _p(check_begin), _p(verdict), _p(status)),
               "cv_partial_merkle_verify")
        return verdict[:ntrees], status[:ntrees]

    # ------------------------------------------------------------ device-resident API
    def verify_device(self, device: int, n: int, d_pk: int, d_sig: int, d_arena: int, d_off: int, d_len: int,
                      d_bitmap: int, d_status: int = 0, stream: int = 0):
        _check(self._lib.cv_ed25519_verify_device(self._h, device, n, d_pk, d_sig, d_arena, d_off, d_len, d_bitmap,
                                                  d_status or None, stream or None), "cv_ed25519_verify_device")

    def verify_device_timed(self, device: int, n: int, d_pk: int, d_sig: int, d_arena: int, d_off: int, d_len: int,
                            d_bitmap: int, stream: int = 0) -> Tuple[float, float, float]:
        """Synchronous verify; returns three kernel durations in ms (HIP events): (scalars, points,
        hs_straus) for throughput batches, (scalars + point pairs, 0, tri / quad Straus) for latency ones."""
        ms = (ctypes.c_float * 3)()
        _check(self._lib.cv_ed25519_verify_device_timed(self._h, device, n, d_pk, d_sig, d_arena, d_off, d_len,
                                                        d_bitmap, stream or None, ms), "cv_ed25519_verify_device_timed")
        return ms[0], ms[1], ms[2]

    def verify_device_keyed(self, device: int, n: int, nkeys: int, d_keys: int, d_key_index: int, d_sig: int,
                            d_arena: int, d_off: int, d_len: int, d_bitmap: int, d_status: int = 0, stream: int = 0,
                            timed: bool = False):
        """Keyed device batch; with timed=True synchronous, returns (keyprep, hash, comb, finish) ms."""
        ms = (ctypes.c_float * 4)() if timed else None
        _check(self._lib.cv_ed25519_verify_device_keyed(self._h, device, n, nkeys, d_keys, d_key_index, d_sig, d_arena,
                                                        d_off, d_len, d_bitmap, d_status or None, stream or None, ms),
               "cv_ed25519_verify_device_keyed")
        return tuple(ms) if timed else None

    def sign_device(self, device: int, n: int, d_seed: int, d_arena: int, d_off: int, d_len: int, d_pk: int,
                    d_sig: int, stream: int = 0):
        _check(self._lib.cv_ed25519_sign_device(self._h, device, n, d_seed, d_arena, d_off, d_len, d_pk, d_sig,
                                                stream or None), "cv_ed25519_sign_device")

    def merkle_device(self, device: int, ntx: int, nleaves: int, d_arena: int, d_off: int, d_len: int,
                      d_tx_begin: int, d_workspace: int, d_ids: int, d_status: int = 0, stream: int = 0):
        _check(self._lib.cv_merkle_tx_ids_device(self._h, device, ntx, nleaves, d_arena, d_off, d_len, d_tx_begin,
                                                 d_workspace, d_ids, d_status or None, stream or None),
               "cv_merkle_tx_ids_device")

    def calibrate(self, device: int) -> Tuple[float, float]:
        """(v_mad_u64_u32 per second, fe_mul per second) measured on `device` (roofline peak)."""
        a, b = ctypes.c_double(0), ctypes.c_double(0)
        _check(self._lib.cv_calibrate(self._h, device, ctypes.byref(a), ctypes.byref(b)), "cv_calibrate")
        return a.value, b.value

    def calibrate_cycles(self, device: int) -> dict:
        """The v_mad_u64_u32 peak on a cycle basis (cv_calibrate_cycles)."""
        o = (ctypes.c_double * 5)()
        _check(self._lib.cv_calibrate_cycles(self._h, device, o), "cv_calibrate_cycles")
        return {"mac_per_s": o[0], "clock_ghz": o[1], "cycles_per_wave_instr": o[2], "simds": int(o[3]),
                "mac_per_s_at_2p4ghz": o[4]}

    def synchronize(self, device: int):
        _check(self._lib.cv_synchronize(self._h, device), "cv_synchronize")


def dedupe_keys(pk: np.ndarray):
    """The engine's host-side key dedupe (cv_diag_dedupe_keys): (key_index, nkeys) or None when the
    batch would not take the keyed path.  Runs on the host; no device needed."""
    lib = load()
    pk = _u8(pk, 32)
    n = len(pk)
    idx = np.zeros(n, np.uint32)
    nk = ctypes.c_size_t(0)
    rc = lib.cv_diag_dedupe_keys(n, _p(pk), _p(idx), ctypes.byref(nk))
    if rc < 0:
        raise CvError(rc, "cv_diag_dedupe_keys")
    return (idx, int(nk.value)) if rc == 1 else None


def tx_verdicts(bitmap: np.ndarray, tx_sig_begin) -> np.ndarray:
    lib = load()
    tx_sig_begin = np.ascontiguousarray(tx_sig_begin, dtype=np.uint32)
    ntx = tx_sig_begin.shape[0] - 1
    out = np.zeros(max(ntx, 0), np.uint8)
    bitmap = np.ascontiguousarray(bitmap, dtype=np.uint64)
    if bitmap.size == 0:
        bitmap = np.zeros(1, np.uint64)
    _check(lib.cv_tx_verdicts(ntx, _p(bitmap), _p(tx_sig_begin), _p(out)), "cv_tx_verdicts")
    return out


def bitmap_to_bools(bitmap: np.ndarray, n: int) -> np.ndarray:
    bits = np.unpackbits(np.ascontiguousarray(bitmap, dtype="<u8").view(np.uint8), bitorder="little")
    return bits[:n].astype(bool)


_default: Optional[Engine] = None
_default_lock = threading.Lock()


def default_engine() -> Engine:
    """Process-wide engine on all visible GPUs (the JVM shim's "one ctx per process")."""
    global _default
    with _default_lock:
        if _default is None:
            _default = Engine(0)
        return _default
