"""Group commit for per-packet Token calls from many threads.

Reticulum calls ``Token`` one packet at a time and synchronously: every
interface's reader thread decrypts the packets it hands to Transport
(``RNS/Interfaces/TCPInterface.py:175,294`` -> ``Transport.inbound`` ->
``Link.receive`` -> ``Link.decrypt``, ``RNS/Link.py:1175-1182``), and
application, Resource and Channel threads encrypt (``RNS/Link.py:1161-1173``,
``RNS/Identity.py:829-830``).  Each such call through ``reticulum_amd.Token``
is one GPU round trip (≈50-65 µs at 500 B), so a node with
many busy interfaces is bound by round trips, not by the kernels.

``CoalescingToken`` has ``Token``'s surface and semantics but hands its calls
to a process-wide ``Coalescer``, which runs them as group commits: the first
caller to arrive becomes a leader and runs every call queued at that moment
as one batch (one ``rt_encrypt_host`` / ``rt_decrypt_host`` /
``rt_verify_host`` per operation and key length, indexing a device table of
the keys seen so far), while the calls that arrive during it queue for the
next leader; up to four leaders run at once, one per staging lane of the
host entry points.  An uncontended call is its own batch of one (no timer,
no helper thread, no added latency); under contention the batch grows with
the number of waiting threads.  Results and exceptions are per call and equal
to ``Token``'s (the same status-to-message mapping, ``Token.py:77-114``).
"""
import ctypes
import os
import threading

import numpy as np

from . import _native
from .token import AES, KeySet, RT_ST_OK, Token, status_message

_ENC, _DEC, _VER = 0, 1, 2


class _Call:
    __slots__ = ("op", "token", "key", "data", "result", "error", "done", "batch", "ev")

    def __init__(self, op, token, data):
        self.op, self.token, self.key, self.data = op, token, token._key, data
        self.result = self.error = self.batch = None
        self.done = False
        self.ev = threading.Event()


class Coalescer:
    """Group-commit executor for Token calls on one device (see module doc).

    Up to ``leaders`` batches run at once (the host entry points have four
    staging lanes, ``token_capi.hip``).  A call that finds a free leader slot
    runs every call queued at that moment (at most ``max_batch``); a leader
    that finishes hands the calls queued meanwhile, as one batch, to the
    first of them, whose thread then leads it (its slot passes on, no thread
    is woken but the batch's own).  A batch of one runs as the plain
    ``Token`` call (its own key set); larger batches index a device table of
    the keys seen so far, one per key length, rebuilt only when a batch
    brings a key it does not hold (at most ``max_keys``; past that the table
    restarts from the batch's keys), so a steady set of links costs no key
    setup per batch.  ``stats`` counts calls, batches (calls / batches = the
    mean batch) and key-table builds."""

    def __init__(self, device=None, max_batch=16384, leaders=4, max_keys=65536):
        self.device = device
        self.max_batch = max_batch
        self.max_leaders = leaders
        self.max_keys = max_keys
        self._lock = threading.Lock()
        self._queue = []
        self._leaders = 0
        self._tables = {}                    # key length -> (KeySet, {key: index})
        self._table_lock = threading.Lock()
        self.stats = {"calls": 0, "batches": 0, "key_tables": 0}

    def _take(self):
        batch = self._queue[:self.max_batch]
        del self._queue[:len(batch)]
        return batch

    def run(self, op, token, data):
        c = _Call(op, token, data)
        with self._lock:
            self._queue.append(c)
            batch = None
            if self._leaders < self.max_leaders:
                self._leaders += 1
                batch = self._take()
        if batch is None:
            c.ev.wait()                      # done, or handed a batch to lead
            batch = None if c.done else c.batch
        if batch is not None:
            try:
                self._execute(batch)
            finally:
                with self._lock:
                    for b in batch:
                        b.done = True
                    self.stats["calls"] += len(batch)
                    self.stats["batches"] += 1
                    nxt = self._take() if self._queue else None
                    if nxt:
                        nxt[0].batch = nxt        # the slot passes to the first waiting call
                    else:
                        self._leaders -= 1
                for b in batch:
                    if b is not c:
                        b.ev.set()
                if nxt:
                    nxt[0].ev.set()
        if c.error is not None:
            raise c.error
        return c.result

    def _table(self, key_len, keys):
        """The key table holding every key of ``keys`` and each key's index."""
        with self._table_lock:
            ks, index = self._tables.get(key_len, (None, {}))
            new = [k for k in dict.fromkeys(keys) if k not in index]
            if new or ks is None:
                base = list(index) if len(index) + len(new) <= self.max_keys else []
                known = set(base)
                all_keys = base + [k for k in dict.fromkeys(keys) if k not in known]
                index = {k: i for i, k in enumerate(all_keys)}
                ks = KeySet(all_keys, device=self.device)
                self._tables[key_len] = (ks, index)
                self.stats["key_tables"] += 1
            return ks, index

    def _execute(self, batch):
        if len(batch) == 1:                  # uncontended: the plain Token call
            c = batch[0]
            try:
                c.result = (Token.encrypt, Token.decrypt, Token.verify_hmac)[c.op](c.token, c.data)
            except Exception as exc:
                c.error = exc
            return
        groups = {}
        for c in batch:
            groups.setdefault((c.op, len(c.key)), []).append(c)
        for (op, klen), calls in groups.items():
            try:
                self._run_group(op, klen, calls)
            except Exception as exc:             # a library error fails the group's calls, not the leader
                for c in calls:
                    c.error = exc

    def _run_group(self, op, klen, calls):
        ks, index = self._table(klen, [c.key for c in calls])
        n = len(calls)
        lib = ks._lib
        kidx = np.fromiter((index[c.key] for c in calls), dtype=np.uint32, count=n)
        lens = np.fromiter((len(c.data) for c in calls), dtype=np.uint32, count=n)
        off = np.zeros(n, dtype=np.uint64)
        np.cumsum(lens[:-1], out=off[1:])
        buf = b"".join(c.data for c in calls) or b"\0"
        vp = ctypes.c_void_p
        if op == _ENC:
            tl = (16 + 16 * (lens.astype(np.uint64) // 16 + 1) + 32)
            toff = np.zeros(n, dtype=np.uint64)
            np.cumsum(tl[:-1], out=toff[1:])
            out = ctypes.create_string_buffer(int(tl.sum()))
            _native.check(lib.rt_encrypt_host(ks._ptr, buf, off.ctypes.data_as(vp), lens.ctypes.data_as(vp),
                                              kidx.ctypes.data_as(vp), os.urandom(16 * n),   # fresh IVs, Token.py:89
                                              out, toff.ctypes.data_as(vp), n))
            raw = out.raw
            for c, o, t in zip(calls, toff.tolist(), tl.tolist()):
                c.result = raw[o:o + t]
        elif op == _DEC:
            cap = np.where(lens > 48, lens.astype(np.int64) - 48, 0).astype(np.uint64)
            poff = np.zeros(n, dtype=np.uint64)
            np.cumsum(cap[:-1], out=poff[1:])
            out = ctypes.create_string_buffer(max(int(cap.sum()), 1))
            olen = np.zeros(n, dtype=np.uint32)
            status = np.zeros(n, dtype=np.int32)
            _native.check(lib.rt_decrypt_host(ks._ptr, buf, off.ctypes.data_as(vp), lens.ctypes.data_as(vp),
                                              kidx.ctypes.data_as(vp), out, poff.ctypes.data_as(vp),
                                              olen.ctypes.data_as(vp), status.ctypes.data_as(vp), n))
            raw = out.raw
            for c, o, m, st in zip(calls, poff.tolist(), olen.tolist(), status.tolist()):
                if st == RT_ST_OK:
                    c.result = raw[o:o + m]
                else:                             # BAD_PAD reports the pad byte in olen
                    c.error = ValueError(status_message(st, len(c.data), m))
        else:
            status = np.zeros(n, dtype=np.int32)
            _native.check(lib.rt_verify_host(ks._ptr, buf, off.ctypes.data_as(vp), lens.ctypes.data_as(vp),
                                             kidx.ctypes.data_as(vp), status.ctypes.data_as(vp), n))
            for c, st in zip(calls, status.tolist()):
                c.result = st == RT_ST_OK


_coalescers = {}
_coalescers_lock = threading.Lock()


def coalescer(device=None):
    """The process-wide Coalescer of ``device``."""
    with _coalescers_lock:
        c = _coalescers.get(device)
        if c is None:
            c = _coalescers[device] = Coalescer(device)
        return c


class CoalescingToken(Token):
    """``Token`` whose calls are group-committed with other threads' calls
    (see module doc).  Same constructor, errors and results as ``Token``
    (``Token.py:40-114``); batch extensions as ``Token``."""

    def __init__(self, key=None, mode=AES, device=None):
        super().__init__(key, mode=mode, device=device)
        self._coalescer = coalescer(device)

    def verify_hmac(self, token):                               # Token.py:77-84
        if len(token) <= 32:
            raise ValueError("Cannot verify HMAC on token of only " + str(len(token)) + " bytes")
        return self._coalescer.run(_VER, self, bytes(token))

    def encrypt(self, data=None):                               # Token.py:87-97
        if not isinstance(data, bytes):
            raise TypeError("Token plaintext input must be bytes")
        return self._coalescer.run(_ENC, self, data)

    def decrypt(self, token=None):                              # Token.py:100-114
        if not isinstance(token, bytes):
            raise TypeError("Token must be bytes")
        if len(token) <= 32:
            raise ValueError("Cannot verify HMAC on token of only " + str(len(token)) + " bytes")
        return self._coalescer.run(_DEC, self, token)
